"""rocprofv3 target: build one config's scene, then render it N times (same launches bench.py times)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
s, p, W, H, desc = R.build_config(cfg)
ctx = R.Context(s)
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
for _ in range(n):
    img, st = ctx.render(cam, p, W, H)
print(cfg, "rays", st.rays, "kernel_ms", st.kernel_ms, flush=True)
