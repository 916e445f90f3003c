"""Developer tool: per-query traversal work (node visits, triangle tests) of the persistent kernel
for each BVH width, from the counting render.  Usage: python tools/query_stats.py [C2 C3 ...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

cfgs = [a for a in sys.argv[1:] if a.startswith("C")] or ["C2", "C3", "C4", "C5"]
widths = ["2", "4", "8"]
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    for bw in widths:
        os.environ["RT_BVH"] = bw
        ctx = R.Context(s)
        R.set_counting(False)
        ctx.render(cam, p, W, H)
        _, st0 = ctx.render(cam, p, W, H)
        R.set_counting(True)
        _, st = ctx.render(cam, p, W, H)
        R.set_counting(False)
        node_b = 64 if bw == "2" else 128
        print(f"{cfg} bvh{bw}: rays={st.rays} nodes/ray={st.node_visits / st.rays:.2f} "
              f"tris/ray={st.tri_tests / st.rays:.2f} hits={st.hits} node_MB={st.node_visits * node_b / 1e6:.0f} "
              f"ms={st0.kernel_ms:.2f} ms_count={st.kernel_ms:.2f}", flush=True)
        ctx.close()
