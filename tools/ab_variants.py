"""Developer tool: A/B of the compiled kernel variants and drain / refill options in ONE process on
one GPU, rounds interleaved so clock drift hits every arm alike.  Per config: median kernel ms of a
single frame and of a V-view turntable batch (rt_render_views_device), per arm.
Usage: python tools/ab_variants.py [C3 C4 ...] [--views V] [--rounds N] [--arms name:k=v,k=v ...] [--lib SO]
(keys are rt_ctx_set_option options, e.g. 6=3 is RT_OPT_VARIANT 3; default arms: every compiled variant)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
import numpy as np  # noqa: E402

import rt_amd as R  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("configs", nargs="*", default=["C3"])
ap.add_argument("--views", type=int, default=16)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--arms", nargs="*", default=None)
ap.add_argument("--lib", default=None, help="another build of librt_amd.so (A/B of two builds: one run each)")
ap.add_argument("--band-count", type=int, default=1,
                help="render rank 0's share of an N-GPU band split (bench.py --gpus N): the per-GPU launch of N GPUs")
args = ap.parse_args()
if args.lib:
    R.LIB_PATH = os.path.abspath(args.lib)

DEFAULTS = {R.OPT_KERNEL: 0, R.OPT_VARIANT: -1, R.OPT_COOP: -1, R.OPT_COOP_MAX: 0, R.OPT_REFILL: 0, R.OPT_FAN: 1, R.OPT_INTERLEAVE: -1, R.OPT_FAN_CAP: 0, R.OPT_DUAL_STEP: -1, R.OPT_OPAQUE: -1, R.OPT_CENTRE_FIRST: -1, R.OPT_TREE: -1, R.OPT_INTERLEAVE_TAIL: 0, R.OPT_WAVEFRONT: -1, R.OPT_WF_BUILD: 0, R.OPT_WF_STREAMS: 0, R.OPT_PRIO: -1, R.OPT_WF_CHUNK: 0}


def parse(a):
    name, kv = a.split(":", 1) if ":" in a else (a, "")
    return name, {int(k): int(v) for k, v in (x.split("=") for x in kv.split(",") if x)}


for cfg in args.configs:
    s, p, W, H, desc = R.build_config(cfg)
    ctx = R.Context(s)
    df = ctx.info()["tri_records"] >= 65536
    if args.arms:
        arms = [parse(a) for a in args.arms]
    else:
        vs = R.DF_VARIANTS if df else R.WT_VARIANTS
        arms = [(f"v{v}", {R.OPT_VARIANT: v}) for v in vs]
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    import torch

    cams = R.turntable_cameras(args.views, R.aspect_of(W, H))
    BC = args.band_count
    buf = torch.zeros(args.views * R.local_band_elems(W, H, 8, BC), dtype=torch.float32, device="cuda")
    res = {n: {"frame": [], "batch": []} for n, _ in arms}
    rays = {}
    sums = {}
    for r in range(args.rounds + 1):
        for name, opts in arms:
            for k, v in DEFAULTS.items():
                ctx.set_option(k, v)
            for k, v in opts.items():
                ctx.set_option(k, v)
            st1 = ctx.render_device(cam, p, W, H, 8, 0, BC, buf.data_ptr(), None)
            stv = ctx.render_views_device(cams, p, W, H, 8, 0, BC, buf.data_ptr(), None) if args.views > 1 else st1
            if r == 0:  # warm-up round: the rays and a checksum of the batch's bits (arms must agree)
                torch.cuda.synchronize()
                x = buf.view(torch.int32).to(torch.int64)
                sums[name] = (int(x.sum()), int((x * x).sum()))
                del x
                rays[name] = (st1.rays, stv.rays, st1.kernel_name)
                continue
            res[name]["frame"].append(st1.kernel_ms)
            res[name]["batch"].append(stv.kernel_ms)
    for name, _ in arms:
        f = float(np.median(res[name]["frame"]))
        b = float(np.median(res[name]["batch"])) / args.views
        r1, rv, kn = rays[name]
        same = "bits = arm 1" if sums[name] == sums[arms[0][0]] and rays[name][1] == rays[arms[0][0]][1] else \
            "BITS DIFFER from arm 1"
        print(f"{cfg} {name:>10}: frame {f:7.3f} ms ({r1 / f / 1e3:7.1f} Mrays/s)  batch {b:7.3f} ms/frame "
              f"({rv / args.views / b / 1e3:7.1f} Mrays/s)  [{kn}] {same} rays {rv} sum {sums[name][0]:x}.{sums[name][1] & 0xFFFFFFFF:x}",
              flush=True)
    ctx.close()
