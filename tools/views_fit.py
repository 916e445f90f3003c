"""Developer tool: C3 ms/frame against the views per launch (8 / 16 / 32 / 64 / 128; tools/ab_variants.py's
timing, one process) and the fit t = a + b / views (a: the per-frame cost at full occupancy, b: the per-launch
drain).  python tools/views_fit.py [CONFIG]"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
vs, ts = [], []
for v in (8, 16, 32, 64, 128):
    out = subprocess.run([sys.executable, "-u", os.path.join(REPO, "tools", "ab_variants.py"), cfg, "--views", str(v),
                          "--rounds", "3", "--arms", "d:"], capture_output=True, text=True, check=True).stdout
    line = [x for x in out.split("\n") if "batch" in x][-1]
    t = float(line.split("batch")[1].split("ms/frame")[0])
    print(f"{cfg} views {v:4d}: {t:.4f} ms/frame   {line.strip()[:110]}", flush=True)
    vs.append(v)
    ts.append(t)
A = np.stack([np.ones(len(vs)), 1.0 / np.array(vs, float)], axis=1)
(a, b), *_ = np.linalg.lstsq(A, np.array(ts), rcond=None)
print(f"fit: t = {a:.4f} + {b:.3f} / views ms/frame (per-frame cost at full occupancy {a:.4f} ms, drain {b:.3f} ms)")
