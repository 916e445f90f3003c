"""Developer tool: A/B env-selected variants on a turntable VIEW BATCH (bench.py's step) in ONE
process, interleaved rounds, median kernel ms per launch; every variant must give the
bit-identical batch and ray count.
Usage: AB_VIEWS=8 python tools/ab_views.py C3 base: r32:RT_REFILL=32 nocoop:RT_COOP=0"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

args = sys.argv[1:]
cfgs = [a for a in args if a.startswith("C") and ":" not in a] or ["C3"]
variants = []
keys = set()
for a in args:
    if ":" in a:
        name, kv = a.split(":", 1)
        env = dict(x.split("=") for x in kv.split(",") if x)
        keys |= set(env)
        variants.append((name, env))
rounds = int(os.environ.get("AB_ROUNDS", "3"))
V = int(os.environ.get("AB_VIEWS", "8"))
import torch  # noqa: E402

for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cams = R.turntable_cameras(V, R.aspect_of(W, H))
    n = R.local_band_elems(W, H, 8, 1)
    buf = torch.zeros(V * n, dtype=torch.float32, device="cuda")
    res = {nm: [] for nm, _ in variants}
    ref = None
    ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
    for r in range(rounds):
        order = variants[r % len(variants):] + variants[:r % len(variants)]
        for nm, env in order:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            for _ in range(2):
                st = ctx.render_views_device(cams, p, W, H, 8, 0, 1, buf.data_ptr(), None)
                res[nm].append(st.kernel_ms)
            torch.cuda.synchronize()
            img = buf.cpu().numpy()
            if ref is None:
                ref = (img.tobytes(), st.rays)
            elif (img.tobytes(), st.rays) != ref:
                print(f"{cfg} {nm}: MISMATCH vs first variant", flush=True)
    for nm, _ in variants:
        print(f"{cfg} V={V} {nm:>10}: median {np.median(res[nm]):.3f} ms/launch  "
              f"{np.median(res[nm]) / V:.3f} ms/frame", flush=True)
