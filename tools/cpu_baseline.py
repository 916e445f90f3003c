"""BASELINE.md's CPU baseline in full, on the GPU box's host cores (run it there: gpurun -- python
tools/cpu_baseline.py --out gpurun_out/cpu_baseline.json).

The reference algorithm as restated by oracle/ref_cpu.cpp (test infrastructure; g++ -O2 -fopenmp) timed on
BASELINE.md's samples: C1 and C2 on the whole frame, C3-C5 on the first 4 096 pixels of the seed-12345
permutation of the frame, rays (intersect() calls: primary, secondary and shadow segments) counted exactly.
Each config runs single-threaded and on every host thread this process may use (OMP_NUM_THREADS on the box),
with useBVH=false (the reference default, src/main.cpp:60) and useBVH=true.  bench.py's cpu_baseline leg is
the bounded-time version of the same measurement for the bench line.

    python tools/cpu_baseline.py [--configs C1,C2,C3,C4,C5] [--pixels 4096] [--out FILE]
"""
import argparse
import json
import os
import platform
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

SAMPLED = {"C3", "C4", "C5"}  # "C3-C5 are timed on a fixed sample of 4096 pixels"


def run(config, pixels, threads_all, seed=12345, log=print):
    import oracle as O
    import rt_amd as R

    scene, prm, W, H, desc = R.build_config(config)
    orc = O.Oracle(scene)
    order = np.random.default_rng(seed).permutation(W * H)
    if config in SAMPLED:
        order = order[:pixels]
    out = {"config": config, "workload": desc, "resolution": f"{W}x{H}",
           "sample": (f"first {len(order)} pixels of the seed-{seed} permutation" if config in SAMPLED
                      else "whole frame"), "legs": {}}
    for bvh in (0, 1):
        p = R.rt_params.from_buffer_copy(prm)
        p.use_bvh = bvh
        for threads in (1, threads_all):
            O.set_threads(threads)
            orc.render_pixels(p, W, H, np.zeros((threads, 2), np.int32))  # start the thread team untimed
            rays, done = 0, 0
            chunk = max(256, 64 * threads)
            t0 = time.perf_counter()
            last = t0
            while done < len(order):
                sel = order[done:done + chunk]
                xy = np.stack([sel % W, sel // W], axis=1).astype(np.int32)
                _, r = orc.render_pixels(p, W, H, xy)
                rays += int(r.sum())
                done += len(sel)
                if time.perf_counter() - last > 30:  # a progress line for long legs
                    last = time.perf_counter()
                    log(f"  {config} bvh{bvh} {threads}t: {done}/{len(order)} pixels, {last - t0:.0f} s", flush=True)
            dt = time.perf_counter() - t0
            key = f"{'1core' if threads == 1 else 'allcore'}_bvh{bvh}"
            out["legs"][key] = {"Mrays_per_s": rays / dt / 1e6, "threads": threads, "pixels": done, "rays": rays,
                                "seconds": round(dt, 3)}
            log(f"{config} {key}: {rays} rays in {dt:.2f} s = {rays / dt / 1e6:.4g} Mrays/s", flush=True)
    return out


def main():
    from bench import _cpu_model, host_threads

    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="C1,C2,C3,C4,C5")
    ap.add_argument("--pixels", type=int, default=4096)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    threads_all = host_threads()
    res = {"host": {"cpu": _cpu_model(), "os_cpu_count": os.cpu_count(), "threads_used_all": threads_all,
                    "python": platform.python_version(),
                    "note": "oracle/ref_cpu.cpp (restatement of the reference CPU path, g++ -O2 -fopenmp); "
                            "threads_used_all = OMP_NUM_THREADS of this box (its CPU share), not os.cpu_count()"},
           "configs": []}
    for c in args.configs.split(","):
        res["configs"].append(run(c.strip(), args.pixels, threads_all))
    text = json.dumps(res, indent=1)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
