"""rocprofv3 target: build one config's scene, then render it N times -- the same launches bench.py
times: one frame (views = 1) or a turntable batch of V views in one launch (bench.py --views V), every pixel
stored in its setPixel place (rt_render_views_image_device).

    python tools/prof_target.py CONFIG N [VIEWS]      (PT_OPTS="16=1" selects render-path options; PT_LIB=path another
                                                       build of the library)
"""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R
if os.environ.get("PT_LIB"):  # another build of the library (developer A/B of builds under the profiler)
    R.LIB_PATH = os.path.abspath(os.environ["PT_LIB"])
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
views = int(sys.argv[3]) if len(sys.argv) > 3 else 1
s, p, W, H, desc = R.build_config(cfg)
ctx = R.Context(s)
# PT_OPTS="k=v,k=v": rt_ctx_set_option settings (developer A/B of render paths under the profiler)
for kv in filter(None, os.environ.get("PT_OPTS", "").split(",")):
    k, v = kv.split("=")
    ctx.set_option(int(k), int(v))
if views == 1:
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    for _ in range(n):
        img, st = ctx.render(cam, p, W, H)
else:
    import torch
    cams = R.turntable_cameras(views, R.aspect_of(W, H))
    buf = torch.zeros(views * W * H * 3, dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    for _ in range(n):
        st = ctx.render_views_image_device(cams, p, W, H, buf.data_ptr(), None)
    torch.cuda.synchronize()
print(cfg, "views", views, "rays", st.rays, "kernel_ms", st.kernel_ms, flush=True)
