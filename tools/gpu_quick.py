"""Quick GPU parity sweep (developer tool): every config at a small size vs the CPU oracle."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import numpy as np  # noqa: E402

import oracle as O  # noqa: E402
import rt_amd as R  # noqa: E402

cases = [("C1", 64, 64, None), ("C2", 64, 48, None), ("C3", 96, 54, (200, 80)), ("C4", 64, 36, (200, 80)),
         ("C5", 96, 54, None)]
if len(sys.argv) > 1:
    cases = [c for c in cases if c[0] in sys.argv[1:]]
for name, W, H, uv in cases:
    s, p, _, _, desc = R.build_config(name, dragon_uv=uv)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    ctx = R.Context(s)
    img, st = ctx.render(cam, p, W, H)
    t = time.time()
    ref, rays = O.Oracle(s).render(p, W, H)
    d = np.abs(img - ref)
    bad = np.argwhere(d.reshape(-1, 3).max(axis=1) > 1e-5).ravel()
    print(f"{name} {W}x{H} {ctx.info()} rays gpu={st.rays} oracle={rays} Linf={d.max():.3g} "
          f"bad_px={len(bad)} gpu_ms={st.kernel_ms:.3f} oracle_s={time.time() - t:.2f}", flush=True)
    for i in bad[:5]:
        y = H - 1 - i // W
        print("   px", i % W, y, img.reshape(-1, 3)[i], ref.reshape(-1, 3)[i])
