"""Developer tool: the wavefront path (RT_OPT_WAVEFRONT 1) against the opaque megakernel on one batch: ray
counts, counted hits, the wavefront's hits per level, and the images bit for bit.

    python tools/wf_check.py [CONFIG] [VIEWS] [WxH]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import rt_amd as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
views = int(sys.argv[2]) if len(sys.argv) > 2 else 8
s, p, W, H, _ = R.build_config(cfg)
if len(sys.argv) > 3:
    W, H = (int(x) for x in sys.argv[3].split("x"))
ctx = R.Context(s)
cams = R.turntable_cameras(views, R.aspect_of(W, H))
out = {}
for name, wf in (("mk", 0), ("wf", 1)):
    ctx.set_option(R.OPT_WAVEFRONT, wf)
    buf = torch.full((views * W * H * 3,), -7.0, dtype=torch.float32, device="cuda")
    st = ctx.render_views_image_device(cams, p, W, H, buf.data_ptr(), None)
    R.set_counting(True)
    cbuf = torch.zeros_like(buf)
    cst = ctx.render_views_image_device(cams, p, W, H, cbuf.data_ptr(), None)
    R.set_counting(False)
    dbg = ctx.debug_counters(50)
    torch.cuda.synchronize()
    img = buf.cpu().numpy()
    out[name] = img
    print(f"{cfg} {views}v {W}x{H} {name}: rays {st.rays} (counting {cst.rays}), hits {cst.hits}, nodes {cst.node_visits}, "
          f"tris {cst.tri_tests}, kernel {st.kernel_ms:.3f} ms" + (f", wf hits/level {[int(x) for x in dbg[32:40]]}" if wf else ""),
          flush=True)
a, b = out["mk"], out["wf"]
diff = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
print(f"images identical: {len(diff) == 0} ({len(diff)} floats differ; untouched wf floats {int(np.sum(b == -7.0))})", flush=True)
if len(diff):
    px = diff // 3
    print("first differing pixels (view, row, col):", [(int(q // (W * H)), int(q % (W * H) // W), int(q % W)) for q in px[:8]])
    print("mk:", a[diff[:6]], "wf:", b[diff[:6]])
ctx.close()
