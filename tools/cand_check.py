"""Developer tool: a candidate librt_amd.so (build/new_librt.so) renders the bench step (C3 1920x1080, 64 views
in one launch), the C3 single frame and a C2 frame (whole-traversal kernel) bit-identically to the in-tree
library; each library in its own process."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r'''
import sys, hashlib, numpy as np
sys.path.insert(0, "raytracer-group27_amd")
import rt_amd as R, torch
if len(sys.argv) > 1: R.LIB_PATH = sys.argv[1]
h = hashlib.sha256()
for cfg in ("C3", "C2"):
    s, p, W, H, _ = R.build_config(cfg)
    ctx = R.Context(s)
    if len(sys.argv) > 2:
        for kv in sys.argv[2].split(","):
            k, v = kv.split("=")
            ctx.set_option(int(k), int(v))
    img, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), p, W, H)
    h.update(img.tobytes()); h.update(str(st.rays).encode())
    if cfg == "C3":
        cams = R.turntable_cameras(64, R.aspect_of(W, H))
        buf = torch.zeros(64 * R.local_band_elems(W, H, 8, 1), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        st = ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
        h.update(buf.cpu().numpy().tobytes()); h.update(str(st.rays).encode())
    ctx.close()
print(h.hexdigest())
'''
out = []
for lib in (None, os.path.join(REPO, "raytracer-group27_amd", "build", "new_librt.so")):
    extra = [lib, os.environ["CAND_OPTS"]] if lib and os.environ.get("CAND_OPTS") else ([lib] if lib else [])
    r = subprocess.run([sys.executable, "-c", CODE] + extra, cwd=REPO, capture_output=True, text=True)
    if r.returncode:
        print(r.stderr[-2000:])
        sys.exit(1)
    out.append(r.stdout.strip().splitlines()[-1])
print("in-tree", out[0])
print("candidate", out[1])
sys.exit(0 if out[0] == out[1] else 1)
