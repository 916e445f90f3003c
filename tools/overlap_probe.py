"""Probe (developer tool): does running two frames' persistent kernels concurrently on two streams
hide the per-frame drain tail?  Sequential frames on one context vs. two host threads, each with
its own context (own job counters / stats) and stream, rendering frames back to back.

    python tools/overlap_probe.py [config] [frames]
"""
import os
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))

import torch  # noqa: E402

import rt_amd as R  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    frames = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    scene, prm, W, H, _ = R.build_config(cfg)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    nctx = 2
    ctxs = [R.Context(scene, device=0) for _ in range(nctx)]
    bufs = [torch.zeros(((H + 7) // 8) * 8 * W * 3, device="cuda") for _ in range(nctx)]
    streams = [torch.cuda.Stream() for _ in range(nctx)]

    def run(i, n, out):
        rays = 0
        for _ in range(n):
            st = ctxs[i].render_device(cam, prm, W, H, 8, 0, 1, bufs[i].data_ptr(), streams[i].cuda_stream)
            rays += st.rays
        out[i] = rays

    for i in range(nctx):
        run(i, 2, {})
    torch.cuda.synchronize()

    out = {}
    t0 = time.perf_counter()
    run(0, frames, out)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"sequential: {frames} frames {dt * 1e3 / frames:.3f} ms/frame {out[0] / dt / 1e6:.1f} Mrays/s", flush=True)

    for k in (2,):
        out = {}
        th = [threading.Thread(target=run, args=(i, frames // k, out)) for i in range(k)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tot = sum(out.values())
        print(f"{k} streams: {frames} frames {dt * 1e3 / frames:.3f} ms/frame {tot / dt / 1e6:.1f} Mrays/s",
              flush=True)
    a = bufs[0].cpu()
    b = bufs[1].cpu()
    print("frames identical:", bool(torch.equal(a, b)), flush=True)


if __name__ == "__main__":
    main()
