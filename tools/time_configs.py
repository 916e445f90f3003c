"""Developer tool: full-size GPU render time + ray count of every BASELINE config (one GPU), one
frame per launch and (TC_VIEWS=V, default 8; 0 = skip) a turntable batch of V views in one launch."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

cfgs = sys.argv[1:] or ["C1", "C2", "C3", "C4", "C5"]
for cfg in cfgs:
    t0 = time.time()
    s, p, W, H, desc = R.build_config(cfg)
    t1 = time.time()
    ctx = R.Context(s)
    t2 = time.time()
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    img, st = ctx.render(cam, p, W, H)
    img, st = ctx.render(cam, p, W, H)
    R.set_counting(True)
    _, cst = ctx.render(cam, p, W, H)
    R.set_counting(False)
    print(f"{cfg} {desc}: load {t1 - t0:.2f}s upload+bvh {t2 - t1:.2f}s kernel {st.kernel_ms:.2f} ms rays {st.rays} "
          f"-> {st.rays / st.kernel_ms / 1e3:.1f} Mrays/s | nodes/ray {cst.node_visits / cst.rays:.1f} "
          f"tris/ray {cst.tri_tests / cst.rays:.1f} hits {cst.hits}", flush=True)
    V = int(os.environ.get("TC_VIEWS", "8"))
    if V > 1:
        import torch
        cams = R.turntable_cameras(V, R.aspect_of(W, H))
        buf = torch.zeros(V * R.local_band_elems(W, H, 8, 1), dtype=torch.float32, device="cuda")
        ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
        vst = ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
        print(f"{cfg} batch of {V} views: kernel {vst.kernel_ms:.2f} ms = {vst.kernel_ms / V:.2f} ms/frame, rays "
              f"{vst.rays} -> {vst.rays / vst.kernel_ms / 1e3:.1f} Mrays/s", flush=True)
        del buf
    ctx.close()
