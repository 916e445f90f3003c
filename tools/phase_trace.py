"""Developer tool: the traversal phases of the slowest waves of one C3 frame (or view batch), from the opaque
kernel's counting build with RT_OPT_WAVE_TRACE 2 (rt_debug_phase_trace): per phase its start, duration, tracing
lanes at its start, traversal iterations and whether it ended in the drain lane groups.
Usage: python tools/phase_trace.py [C3] [views] [waves to show]"""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
views = int(sys.argv[2]) if len(sys.argv) > 2 else 1
show = int(sys.argv[3]) if len(sys.argv) > 3 else 6
s, p, W, H, desc = R.build_config(cfg)
ctx = R.Context(s)
ctx.set_option(R.OPT_WAVE_TRACE, 2)
R.lib().rt_set_counting(1)
if views == 1:
    _, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), p, W, H)
else:
    _, st = ctx.render_views(R.turntable_cameras(views, R.aspect_of(W, H)), p, W, H)
EV = 512
wt = np.zeros(8 * 65536, np.uint64)
nw = R.lib().rt_debug_wave_trace(ctx.h, wt.ctypes.data_as(C.POINTER(C.c_uint64)), 65536)
wt = wt[:8 * nw].reshape(nw, 8).astype(np.int64)
ph = np.zeros(nw * EV * 2, np.uint64)
n = R.lib().rt_debug_phase_trace(ctx.h, ph.ctypes.data_as(C.POINTER(C.c_uint64)), nw)
ph = ph[:n * EV * 2].reshape(n, EV, 2)
t0 = int(wt[:, 0].min())
M40 = (1 << 40) - 1
w0 = (wt[:n, 0] - t0)[:, None]  # the waves' starts
start = ((ph[:, :, 0] & np.uint64(M40)).astype(np.int64) + w0) / 100.0
ntr = ((ph[:, :, 0] >> np.uint64(48)) & np.uint64(127)).astype(np.int64)
end = ((ph[:, :, 1] & np.uint64(M40)).astype(np.int64) + w0) / 100.0
iters = ((ph[:, :, 1] >> np.uint64(40)) & np.uint64((1 << 23) - 1)).astype(np.int64)
coop = (ph[:, :, 1] >> np.uint64(63)).astype(np.int64)
valid = ph[:, :, 1] != 0
dur = np.where(valid, end - start, 0.0)
wend = (wt[:, 1] - t0) / 100.0
print(f"{cfg} {views}v: {st.kernel_name} kernel {st.kernel_ms:.3f} ms, waves {nw}, phases/wave "
      f"{np.percentile(valid.sum(1), [0, 50, 99, 100]).round(0).tolist()}")
print("phase duration us pct (0 50 90 99 99.9 100):", np.percentile(dur[valid], [0, 50, 90, 99, 99.9, 100]).round(1).tolist())
print("phase iterations pct:", np.percentile(iters[valid], [0, 50, 90, 99, 99.9, 100]).round(0).tolist())
print("us per iteration pct:", np.percentile((dur[valid] / np.maximum(1, iters[valid])), [0, 50, 90, 99, 100]).round(2).tolist())
# where the tail goes: the slowest waves' phases after the median wave end
order = np.argsort(-wend)
med = float(np.median(wend))
for w in order[:show]:
    m = valid[w] & (end[w] > med - 50)
    print(f" wave {w}: end {wend[w]:.1f} us, jobs {wt[w, 2]}, dry {(wt[w, 3] - t0) / 100.0 if wt[w, 3] else -1:.1f}")
    for k in np.nonzero(m)[0]:
        print(f"   phase {k:3d}: {start[w, k]:8.1f} .. {end[w, k]:8.1f} us ({dur[w, k]:7.1f}) tracing {ntr[w, k]:2d} "
              f"iters {iters[w, k]:4d}{' lane groups' if coop[w, k] else ''}")

# the jobs that finished last: where they are in the image (job trace word 2 = the pixel id y * W + x)
nj = 1 << 23
jt = np.zeros(3 * nj, np.uint64)
nj = R.lib().rt_debug_job_trace(ctx.h, jt.ctypes.data_as(C.POINTER(C.c_uint64)), nj)
jt = jt[:3 * nj].reshape(nj, 3).astype(np.int64)
done = jt[:, 1] > 0
js = (jt[done, 0] - t0) / 100.0
je = (jt[done, 1] - t0) / 100.0
pix = jt[done, 2] % (W * H)
py, px = pix // W, pix % W
print("job start us pct (0 50 90 99 100):", np.percentile(js, [0, 50, 90, 99, 100]).round(1).tolist())
print("job latency us pct (0 50 90 99 99.9 100):", np.percentile(je - js, [0, 50, 90, 99, 99.9, 100]).round(1).tolist())
late = np.argsort(-je)[:2000]
print(f"the 2000 last jobs: start us pct {np.percentile(js[late], [0, 50, 100]).round(1).tolist()}, latency pct "
      f"{np.percentile((je - js)[late], [0, 50, 100]).round(1).tolist()}")
# coarse map (12 x 8 cells): mean job latency, and the share of the last 2000 jobs
gy, gx = 8, 12
cy, cx = py * gy // H, px * gx // W
lat = je - js
print("mean job latency (us) by image cell (y up: row 0 = bottom of the frame):")
for r in range(gy - 1, -1, -1):
    row = []
    for c in range(gx):
        m = (cy == r) & (cx == c)
        row.append(f"{lat[m].mean():6.0f}" if m.any() else "     -")
    print("  " + " ".join(row))
print("cells of the 2000 last jobs (count):")
cnt = np.zeros((gy, gx), int)
np.add.at(cnt, (cy[late], cx[late]), 1)
for r in range(gy - 1, -1, -1):
    print("  " + " ".join(f"{v:6d}" for v in cnt[r]))
print("mean job start (us) by cell:")
for r in range(gy - 1, -1, -1):
    row = []
    for c in range(gx):
        m = (cy == r) & (cx == c)
        row.append(f"{js[m].mean():6.0f}" if m.any() else "     -")
    print("  " + " ".join(row))
