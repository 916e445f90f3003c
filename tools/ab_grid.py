"""Developer tool: persistent-kernel grid size A/B (blocks per CU) in one process.
Usage: python tools/ab_grid.py C3 C5 g=8,12,16"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np
import rt_amd as R
cfgs = [a for a in sys.argv[1:] if a.startswith("C")] or ["C3", "C5"]
grids = [None]
for a in sys.argv[1:]:
    if a.startswith("g="):
        grids += a[2:].split(",")
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    res = {g: [] for g in grids}
    for _ in range(3):
        for g in grids:
            if g is None:
                os.environ.pop("RT_GRID", None)
            else:
                os.environ["RT_GRID"] = g
            img, st = ctx.render(cam, p, W, H)
            res[g].append(st.kernel_ms)
    print(f"{cfg} rays={st.rays} " + " ".join(f"g{g or 'api'}={np.median(t):.3f}" for g, t in res.items()), flush=True)
    ctx.close()
