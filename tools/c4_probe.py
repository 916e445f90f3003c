"""Developer tool: C4 single-frame kernel time under render options and sample counts."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

s, p, W, H, desc = R.build_config("C4")
ctx = R.Context(s)
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
arms = [("default", {}), ("fan0", {R.OPT_FAN: 0}), ("refill64", {R.OPT_REFILL: 64}), ("refill8", {R.OPT_REFILL: 8}),
        ("coop0", {R.OPT_COOP: 0}), ("v23", {R.OPT_VARIANT: R.DF_BATCH}), ("v23r64", {R.OPT_VARIANT: R.DF_BATCH, R.OPT_REFILL: 64})]
for n in (64, 16, 4):
    q = R.rt_params.from_buffer_copy(p)
    q.sphere_light_ray_count = n
    for name, opts in arms:
        for k, v in {R.OPT_KERNEL: 0, R.OPT_VARIANT: -1, R.OPT_COOP: -1, R.OPT_COOP_MAX: 0, R.OPT_REFILL: 0,
                     R.OPT_FAN: 1, R.OPT_INTERLEAVE: -1, R.OPT_FAN_CAP: 0, R.OPT_DUAL_STEP: -1}.items():
            ctx.set_option(k, v)
        for k, v in opts.items():
            ctx.set_option(k, v)
        ms = []
        for _ in range(3):
            _, st = ctx.render(cam, q, W, H)
            ms.append(st.kernel_ms)
        print(f"samples {n:3d} {name:9s}: {min(ms):8.3f} ms  rays {st.rays}  {st.rays / min(ms) / 1e3:8.1f} Mrays/s",
              flush=True)
