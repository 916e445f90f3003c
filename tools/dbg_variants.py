"""Developer tool: per-variant ray counts and image error vs the oracle on the glossy Cornell scene."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402
from oracle import oracle as O  # noqa: E402
from test_glossy import _cornell  # noqa: E402

s, p = _cornell(R, 10, 0x5EED)
W, H = 48, 27
ctx = R.Context(s)
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
ref, rays = O.Oracle(s).render(p, W, H)
print("oracle rays", rays, flush=True)
arms = [(v, c) for v in R.DF_VARIANTS for c in (-1, 0)]
for v, c in arms:
    ctx.set_option(R.OPT_KERNEL, R.KERNEL_DYNAMIC_FETCH)
    ctx.set_option(R.OPT_VARIANT, v)
    ctx.set_option(R.OPT_COOP, c)
    img, st = ctx.render(cam, p, W, H)
    print(f"v{v} coop{c}: rays {st.rays} maxerr {float(np.max(np.abs(img - ref))):.3g} kernel {st.kernel_name}",
          flush=True)
