"""Developer tool: single-frame kernel ms per config under option sets (rt_ctx_set_option key=value)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

cfgs = [a for a in sys.argv[1:] if ":" not in a] or ["C3", "C4"]
arms = [(a.split(":", 1)[0], {int(k): int(v) for k, v in (x.split("=") for x in a.split(":", 1)[1].split(",") if x)})
        for a in sys.argv[1:] if ":" in a] or [("default", {})]
DEF = {R.OPT_KERNEL: 0, R.OPT_VARIANT: -1, R.OPT_COOP: -1, R.OPT_COOP_MAX: 0, R.OPT_REFILL: 0, R.OPT_FAN: 1,
       R.OPT_INTERLEAVE: -1, R.OPT_FAN_CAP: 0, R.OPT_DUAL_STEP: -1}
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    for name, opts in arms:
        for k, v in {**DEF, **opts}.items():
            ctx.set_option(k, v)
        ms = []
        for _ in range(4):
            _, st = ctx.render(cam, p, W, H)
            ms.append(st.kernel_ms)
        print(f"{cfg} {name:10s}: {min(ms):9.3f} ms  rays {st.rays}  {st.rays / min(ms) / 1e3:8.1f} Mrays/s "
              f"[{st.kernel_name}]", flush=True)
    ctx.close()
