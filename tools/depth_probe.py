"""Developer tool: C3 single-frame kernel time against max_reflection_level (the chain latency of the drain).
Usage: python tools/depth_probe.py [option=value ...]"""
import sys, os, time
sys.path.insert(0, "raytracer-group27_amd")
import numpy as np, rt_amd as R
s, p, W, H, _ = R.build_config("C3")
ctx = R.Context(s)
for a in sys.argv[1:]:  # rt_ctx_set_option k=v
    k, v = a.split("=")
    ctx.set_option(int(k), int(v))
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
for depth in (0, 1, 2, 3, 4):
    pp = R.params(max_reflection_level=depth, glossy_ray_count=1)
    ts = []
    for r in range(8):
        _, st = ctx.render(cam, pp, W, H)
        ts.append(st.kernel_ms)
    print(f"depth {depth}: kernel ms median {np.median(ts[2:]):.3f}  rays {st.rays}", flush=True)
