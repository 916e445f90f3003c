"""Developer tool: A/B the render kernel variants in ONE process (cdna guide rule 24):
tile kernel vs persistent megakernel at WPE 1..4, interleaved rounds, median kernel ms."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

cfgs = [a for a in sys.argv[1:] if a.startswith("C")] or ["C2", "C3", "C4", "C5"]
variants = [("tile", None), ("persistent", "1"), ("persistent", "2"), ("persistent", "3"), ("persistent", "4")]
rounds = 3
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    res = {v: [] for v in variants}
    ref_img = None
    for _ in range(rounds):
        for v in variants:
            os.environ["RT_KERNEL"] = v[0]
            if v[1]:
                os.environ["RT_WPE"] = v[1]
            img, st = ctx.render(cam, p, W, H)
            if ref_img is None:
                ref_img, ref_rays = img, st.rays
            assert st.rays == ref_rays, (v, st.rays, ref_rays)
            assert img.tobytes() == ref_img.tobytes(), v
            res[v].append(st.kernel_ms)
    line = " ".join(f"{v[0][:4]}{v[1] or ''}={np.median(t):.2f}ms" for v, t in res.items())
    best = min(res, key=lambda v: np.median(res[v]))
    print(f"{cfg} rays={ref_rays} {line} best={best} -> {ref_rays / np.median(res[best]) / 1e3:.0f} Mrays/s", flush=True)
    ctx.close()
