"""Developer tool: rt_create phase times (rt_debug_create_ms) for the C3 scene, a few runs."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import torch  # noqa: E402,F401

import rt_amd as R  # noqa: E402

torch.zeros(1, device="cuda")
s, p, W, H, desc = R.build_config(sys.argv[1] if len(sys.argv) > 1 else "C3")
for _ in range(3):
    t0 = time.perf_counter()
    ctx = R.Context(s)
    wall = (time.perf_counter() - t0) * 1e3
    print(f"wall {wall:7.1f} ms  phases (cumulative ms) {' '.join(f'{x:7.1f}' for x in ctx.create_ms())}", flush=True)
    ctx.close()
