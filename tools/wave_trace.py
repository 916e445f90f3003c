"""Developer tool: per-wave timeline of the persistent render kernel (context option RT_OPT_WAVE_TRACE) -- launch
skew, when each wave found the job queue empty, and what it did until it retired (drain
iterations, tracing lanes per iteration, state-machine passes).
Usage: python tools/wave_trace.py C3 [C4 ...]
The opaque-scene kernel fills the drain columns (iterations, lanes, lane-group walks, phase-A passes) in its
counting build only (WT_COUNT=1 -- the shipped build keeps those counters out of its registers)."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

Q = [0, 1, 5, 25, 50, 75, 95, 99, 100]


def pct(x):
    return " ".join(f"{v:.1f}" for v in np.percentile(x, Q))


for cfg in [a for a in sys.argv[1:] if a.startswith("C")] or ["C3"]:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    ctx.set_option(R.OPT_WAVE_TRACE, 1)
    if os.environ.get("WT_COUNT") == "1":
        R.lib().rt_set_counting(1)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    V = int(os.environ.get("WT_VIEWS", "1"))  # > 1: a V-view turntable batch in one launch
    if V > 1:
        import torch
        cams = R.turntable_cameras(V, R.aspect_of(W, H))
        vb = torch.zeros(V * R.local_band_elems(W, H, 8, 1), dtype=torch.float32, device="cuda")
        ctx.render_views_device(cams, p, W, H, 8, 0, 1, vb.data_ptr(), None)
        st = ctx.render_views_device(cams, p, W, H, 8, 0, 1, vb.data_ptr(), None)
    else:
        ctx.render(cam, p, W, H)
        _, st = ctx.render(cam, p, W, H)
    buf = np.zeros(8 * 65536, np.uint64)
    n = R.lib().rt_debug_wave_trace(ctx.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), 65536)
    t = buf[:8 * n].reshape(n, 8).astype(np.int64)
    t0 = t[:, 0].min()
    start, end = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0  # us
    print(f"{cfg}: waves={n} kernel_ms={st.kernel_ms:.3f} span_us={end.max():.1f}", flush=True)
    print("  start us pct " + pct(start))
    print("  end   us pct " + pct(end))
    print(f"  mean lifetime / span = {(end - start).mean() / end.max():.3f}; jobs/wave pct "
          + " ".join(f"{x:.0f}" for x in np.percentile(t[:, 2], [0, 50, 100])))
    dr = t[:, 3] > 0
    if dr.any():
        exh = (t[dr, 3] - t0) / 100.0
        drain = end[dr] - exh
        it = np.maximum(t[dr, 4], 1)
        print("  queue dry us pct " + pct(exh))
        print("  drain us pct     " + pct(drain))
        print("  drain iters pct  " + pct(t[dr, 4]))
        print("  lanes/iter pct   " + pct(t[dr, 5] / it))
        print("  us/iter pct      " + pct(drain / it))
        print("  drain phase-A passes pct " + pct(t[dr, 7]))
        print("  lane-group walks pct " + pct(t[dr, 6]))
        last = np.argsort(end)[-5:]
        for i in last:
            print(f"   last wave {i}: end {end[i]:.1f} dry {(t[i, 3] - t0) / 100.0:.1f} iters {t[i, 4]} "
                  f"lanes/iter {t[i, 5] / max(1, t[i, 4]):.1f} phaseA {t[i, 7]}")
    ctx.close()
