"""Developer tool: A/B render-kernel variants in ONE process (cdna guide rule 24), interleaved
rounds, median kernel ms.  Variants are env settings read per launch by rt_runtime.hip:
RT_KERNEL=tile|persistent, RT_WPE (register cap), RT_BVH (2 = binary, 8 = quantised 8-wide)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

args = sys.argv[1:]
cfgs = [a for a in args if a.startswith("C")] or ["C2", "C3", "C4", "C5"]
specs = [a for a in args if "=" in a]  # e.g. WPE=1,2 BVH=2,8
variants = [{"RT_KERNEL": "tile"}]
wpes = ["2"]
bvhs = ["2", "4", "8"]
for s in specs:
    k, v = s.split("=")
    if k == "WPE":
        wpes = v.split(",")
    if k == "BVH":
        bvhs = v.split(",")
for w in wpes:
    for b in bvhs:
        variants.append({"RT_KERNEL": "persistent", "RT_WPE": w, "RT_BVH": b})
rounds = 3


def name(v):
    if v["RT_KERNEL"] == "tile":
        return "tile"
    return f"w{v['RT_WPE']}b{v['RT_BVH']}"


for cfg in cfgs:
    s, p, W, H, desc = R.build_config(cfg)
    ctxs = {}
    for v in variants:  # the BVH width is fixed when a context is created
        b = v.get("RT_BVH", "2")
        if b not in ctxs:
            os.environ["RT_BVH"] = b
            ctxs[b] = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    res = {name(v): [] for v in variants}
    ref_img = None
    for _ in range(rounds):
        for v in variants:
            os.environ.update(v)
            img, st = ctxs[v.get("RT_BVH", "2")].render(cam, p, W, H)
            if ref_img is None:
                ref_img, ref_rays = img, st.rays
            assert st.rays == ref_rays, (v, st.rays, ref_rays)
            assert img.tobytes() == ref_img.tobytes(), v
            res[name(v)].append(st.kernel_ms)
    line = " ".join(f"{k}={np.median(t):.2f}" for k, t in res.items())
    best = min(res, key=lambda k: np.median(res[k]))
    print(f"{cfg} rays={ref_rays} {line} | best={best} {ref_rays / np.median(res[best]) / 1e3:.0f} Mrays/s", flush=True)
    for c in ctxs.values():
        c.close()
