"""Developer tool: per-job (pixel) latency of one frame from the persistent kernel's job trace
(RT_OPT_WAVE_TRACE): start / end times, queries per job, the slowest jobs and when jobs started.
Usage: python tools/job_trace.py C4 [fan=0|1] [opaque=0|-1] [coop=N] [refill=N] [variant=V]
(the opaque-scene kernel keeps its trace stores out of the shipped build: its trace comes from the counting build)"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C4"
s, p, W, H, desc = R.build_config(cfg)
ctx = R.Context(s)
for a in sys.argv[2:]:
    k, v = a.split("=")
    ctx.set_option({"fan": R.OPT_FAN, "variant": R.OPT_VARIANT, "refill": R.OPT_REFILL, "opaque": R.OPT_OPAQUE,
                    "coop": R.OPT_COOP}[k], int(v))
ctx.set_option(R.OPT_WAVE_TRACE, 1)
cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
_, st = ctx.render(cam, p, W, H)
if "opaque" in st.kernel_name:  # the opaque-scene kernel records its traces in the counting build only
    R.lib().rt_set_counting(1)
    print("(opaque-scene kernel: counting build)")
    ctx.render(cam, p, W, H)
_, st = ctx.render(cam, p, W, H)
nj = 1 << 23
buf = np.zeros(3 * nj, np.uint64)
n = R.lib().rt_debug_job_trace(ctx.h, buf.ctypes.data_as(C.POINTER(C.c_uint64)), nj)
jt = buf[:3 * n].reshape(n, 3).astype(np.int64)
wt = np.zeros(8 * 65536, np.uint64)
nw = R.lib().rt_debug_wave_trace(ctx.h, wt.ctypes.data_as(C.POINTER(C.c_uint64)), 65536)
t0 = int(wt[0:8 * nw:8].min())
done = jt[:, 1] > 0
st_us = (jt[done, 0] - t0) / 100.0
en_us = (jt[done, 1] - t0) / 100.0
lat = en_us - st_us
q = jt[done, 2]
print(f"{cfg}: kernel {st.kernel_ms:.3f} ms, jobs {n}, traced {done.sum()}")
if os.environ.get("JT_SAVE"):  # per-job (start us, end us, queries) for offline analysis
    np.savez_compressed(os.environ["JT_SAVE"], start=((jt[:, 0] - t0) / 100.0).astype(np.float32),
                        end=((jt[:, 1] - t0) / 100.0).astype(np.float32), queries=jt[:, 2].astype(np.int32),
                        done=done, W=W, H=H)
P = [0, 50, 90, 99, 99.9, 100]
print("latency us pct", " ".join(f"{v:.1f}" for v in np.percentile(lat, P)))
print("queries pct   ", " ".join(f"{v:.0f}" for v in np.percentile(q, P)))
print("start us pct  ", " ".join(f"{v:.1f}" for v in np.percentile(st_us, P)))
print("end us pct    ", " ".join(f"{v:.1f}" for v in np.percentile(en_us, P)))
for lo in (1, 2, 30, 60):
    m = q >= lo
    if m.any():
        print(f"  jobs with >= {lo:3d} queries: {m.sum():8d}  latency us median {np.median(lat[m]):9.1f}  "
              f"us/query median {np.median(lat[m] / q[m]):7.2f}")
idx = np.argsort(-lat)[:12]
jobs = np.nonzero(done)[0]
for i in idx:
    print(f"  slow job {jobs[i]:8d}: start {st_us[i]:9.1f} end {en_us[i]:9.1f} latency {lat[i]:9.1f} us, queries {q[i]}")
# time profile: jobs in flight per 1 ms
T = int(en_us.max() / 1000) + 1
for ms in range(0, T, max(1, T // 12)):
    a, b = ms * 1000.0, (ms + 1) * 1000.0
    print(f"  t={ms:3d} ms: started {int(((st_us >= a) & (st_us < b)).sum()):8d}  ended {int(((en_us >= a) & (en_us < b)).sum()):8d}"
          f"  in flight {int(((st_us < a) & (en_us >= a)).sum()):7d}")
