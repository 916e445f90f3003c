import sys, os, time
sys.path.insert(0, "raytracer-group27_amd")
import numpy as np, rt_amd as R
s, p, W, H, _ = R.build_config("C3")
ctx = R.Context(s)
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
for depth in (0, 1, 2, 3, 4):
    pp = R.params(max_reflection_level=depth, glossy_ray_count=1)
    ts = []
    for r in range(8):
        _, st = ctx.render(cam, pp, W, H)
        ts.append(st.kernel_ms)
    print(f"depth {depth}: kernel ms median {np.median(ts[2:]):.3f}  rays {st.rays}", flush=True)
