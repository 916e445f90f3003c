"""Developer tool: per-query node-visit distribution of the wavefront trace kernel (counting build)
and per-iteration trace times.  Usage: python tools/wf_hist.py C3 C4"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

for cfg in [a for a in sys.argv[1:] if a.startswith("C")] or ["C3"]:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    _, st = ctx.render(cam, p, W, H)
    R.set_counting(True)
    _, cst = ctx.render(cam, p, W, H)
    R.set_counting(False)
    c = [int(x) for x in ctx.debug_counters()]
    print(f"{cfg}: rays={cst.rays} nodes/ray={cst.node_visits / cst.rays:.2f} tris/ray={cst.tri_tests / cst.rays:.2f} "
          f"max_nodes={c[10]} hist(<64,<256,<1k,<4k,>=4k)={c[11:16]} frame_ms={st.kernel_ms:.3f} "
          f"trace_ms={st.trace_ms:.3f} launches={st.trace_launches}", flush=True)
    ctx.close()
