"""Developer tool: A/B env-selected kernel variants in ONE process, interleaved rounds, median
kernel ms; every variant must give the bit-identical image and ray count.
Usage: python tools/ab_env.py C3 C5 old:RT_KERNEL=persistent r8:RT_REFILL=8 r16:RT_REFILL=16"""
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
for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    res = {n: [] for n, _ in variants}
    ref = None
    ctx.render(cam, p, W, H)  # warm-up (code object load, scratch)
    for rd in range(rounds):
        order = variants[rd % len(variants):] + variants[:rd % len(variants)]  # rotate: no first-slot bias
        for n, env in order:
            for k in keys:
                os.environ.pop(k, None)
            os.environ.update(env)
            img, st = ctx.render(cam, p, W, H)
            if ref is None:
                ref = (img, st.rays, n)
            same = img.tobytes() == ref[0].tobytes() and st.rays == ref[1]
            if not same:
                print(f"MISMATCH {cfg} {n} vs {ref[2]}: rays {st.rays} vs {ref[1]} "
                      f"Linf {float(np.max(np.abs(img - ref[0]))):.3g}", flush=True)
            res[n].append(st.kernel_ms)
    line = " ".join(f"{k}={np.median(t):.3f}" for k, t in res.items())
    best = min(res, key=lambda k: np.median(res[k]))
    print(f"{cfg} rays={ref[1]} {line} | best={best} {ref[1] / np.median(res[best]) / 1e3:.0f} Mrays/s", flush=True)
    ctx.close()
