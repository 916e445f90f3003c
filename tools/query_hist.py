"""Developer tool: per-query node-visit histogram (counting build) for each config."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R
for cfg in (sys.argv[1:] or ["C2", "C3", "C4", "C5"]):
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    R.set_counting(True)
    img, st = ctx.render(cam, p, W, H)
    R.set_counting(False)
    h = ctx.debug_counters()
    print(f"{cfg} rays={st.rays} nodes/ray={st.node_visits/st.rays:.1f} hist(<16,<64,<256,<1k,<4k,>=4k)={list(map(int,h[8:14]))} "
          f"max_nodes={int(h[14])} max_tris={int(h[15])} ms={st.kernel_ms:.2f}", flush=True)
    ctx.close()
