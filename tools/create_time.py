"""Developer tool: rt_create phase times (rt_debug_create_ms) for a config, a few runs per build mode.
Usage: python tools/create_time.py [CONFIG] [MODES] (modes: comma list of 0 auto, 1 host, 2 GPU)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import torch  # noqa: E402,F401

import rt_amd as R  # noqa: E402

torch.zeros(1, device="cuda")
s, p, W, H, desc = R.build_config(sys.argv[1] if len(sys.argv) > 1 else "C3")
modes = [int(m) for m in (sys.argv[2] if len(sys.argv) > 2 else "1,2").split(",")]
for mode in modes:
    R.set_build_mode(mode)
    for _ in range(3):
        t0 = time.perf_counter()
        ctx = R.Context(s)
        wall = (time.perf_counter() - t0) * 1e3
        print(f"mode {mode} wall {wall:7.1f} ms  phases (cumulative ms) "
              f"{' '.join(f'{x:7.1f}' for x in ctx.create_ms())}  {ctx.build_info()}", flush=True)
        ctx.close()
R.set_build_mode(0)
