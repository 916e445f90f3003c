"""Developer probe: how many queries of a render walk every triangle record (a direction whose squared length is
not within 4e-6 of 1 takes trav_init_q's exhaustive path), counted by the opaque kernel's counting build
(debug counter 28), and the directions' lengths of a few of them.
Usage: python tools/exh_count.py C3 [views]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
views = int(sys.argv[2]) if len(sys.argv) > 2 else 1
s, p, W, H, desc = R.build_config(cfg)
ctx = R.Context(s)
ctx.set_option(R.OPT_WAVE_TRACE, 1)  # the per-query counters are kept only with the wave trace on
R.lib().rt_set_counting(1)
if views == 1:
    _, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), p, W, H)
else:
    _, st = ctx.render_views(R.turntable_cameras(views, R.aspect_of(W, H)), p, W, H)
c = ctx.debug_counters(32)
print(f"{cfg} {views}v: {st.kernel_name} rays {st.rays} kernel {st.kernel_ms:.3f} ms; exhaustive queries {c[28]}"
      f" ({c[28] / max(1, st.rays):.2e} of rays); longest query: {c[29]} node visits, {c[30]} records; queries"
      f" with > 512 node visits {c[31]} (the drain lane groups' walks are not in these)")
