"""bench.py -- Mrays/s of the MI355X ray tracer on BASELINE.json's 1920x1080 workload.

Workload (config.workload): C3 = dragon proxy (800 000 triangles), 1920x1080,
one point light, hard shadows + mirror recursion depth 4 (BASELINE.json configs[2]).  One step
renders a batch of --views full frames (default 16: a turntable of the scene, 22.5 degrees apart) in
ONE launch of the persistent kernel (rt_render_views_device), each frame un-permuted into its own
Screen::m_textureData image; every rank renders its own batch (weak scaling, no collective on the
data path).  --views 1 renders one frame per step; --partition bands splits one frame over the
ranks in interleaved 8-row bands, gathered over RCCL (torch.distributed "nccl") and un-permuted
on rank 0.  Inputs (scene, BVH) are resident in HBM before timing starts.  The JSON also carries
`single_frame`: the default view rendered alone (one launch per frame), timed the same way.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--views V] [--no-cpu-baseline]

Prints ONE JSON line on rank 0.  `value` = rays (intersect() calls) of all ranks / max-rank time.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))

import numpy as np  # noqa: E402

METRIC = "Mrays/s (primary+shadow+secondary) at 1920×1080; fraction of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BAND_ROWS = 8
DEFAULT_VIEWS = 16  # frames per step: a 16-view turntable (22.5 deg apart) of the C3 scene in one launch


def algorithmic_bytes(st, pixels):
    """one node record per node visit (64 B BVH2, 128 B quantised BVH8 -- the
    structure the kernel walks), 64 B per triangle record, 68 B per shaded hit (3 normals +
    material), 12 B per pixel written."""
    return int(st.node_bytes or 64) * st.node_visits + 64 * st.tri_tests + 68 * st.hits + 12 * pixels


def kernel_name(ntri):
    """Name of the dominant kernel as rocprofv3 lists it (rt_runtime.hip: RT_KERNEL / RT_WPE / RT_BVH;
    by default whole-traversal refill below 65 536 triangles, dynamic fetch above)."""
    k = os.environ.get("RT_KERNEL")
    if k == "tile":
        return "rt::render_kernel<false>"
    wpe = 1 if os.environ.get("RT_WPE") == "1" else 2
    bw = os.environ.get("RT_BVH", "8")
    bw = bw if bw in ("2", "4") else "8"
    if k == "wavefront":
        return f"rt::wf_trace_kernel<false, 4, {bw}>"
    # wpe 2 without textures launches the TEX=false specialisation (no texture code); the
    # persistent kernel has it for the 8-wide BVH only
    if k == "persistent" or (k != "df" and ntri < 65536) or bw == "2":
        tex = ", false" if (wpe == 2 and bw == "8") else ""
        return f"rt::persistent_kernel<false, {wpe}, {bw}{tex}>"
    tex = ", false" if wpe == 2 else ""
    return f"rt::persistent_df_kernel<false, {wpe}, {bw}{tex}>"


def cpu_baseline(config, budget_s=12.0, seed=12345):
    """Reference algorithm (oracle/ref_cpu.cpp: brute-force primary/secondary rays, depth-4 BVH for
    shadow rays) timed single-threaded on a fixed pseudo-random pixel sample of the same frame."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    scene, prm, W, H, _ = R.build_config(config)
    O.set_threads(1)
    orc = O.Oracle(scene)
    rng = np.random.default_rng(seed)
    order = rng.permutation(W * H)
    rays = 0
    npx = 0
    t0 = time.perf_counter()
    chunk = 4
    while time.perf_counter() - t0 < budget_s and npx < len(order):
        sel = order[npx:npx + chunk]
        xy = np.stack([sel % W, sel // W], axis=1)
        _, r = orc.render_pixels(prm, W, H, xy)
        rays += int(r.sum())
        npx += len(sel)
    dt = time.perf_counter() - t0
    return {"value": rays / dt / 1e6, "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"{npx} pseudo-random pixels (seed {seed}) of {config} {W}x{H}, {rays} rays in {dt:.1f} s, "
                      f"OMP_NUM_THREADS=1, host CPU: {_cpu_model()}"}


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc(config, kernel):
    """HBM bytes per render launch from the committed rocprofv3 --pmc summary of the same kernel
    (tools/profile.sh + tools/pmc_summary.py --latest), or None."""
    p = os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("config") == config and kernel in (d.get("kernel") or ""):
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-single-frame", action="store_true",
                    help="skip the single-frame latency record (profiling runs: one kernel shape only)")
    ap.add_argument("--partition", choices=("frames", "bands"), default="frames",
                    help="N>1: frames = every rank renders whole frames of its own (weak scaling, no collective "
                         "on the data path); bands = one frame split into interleaved 8-row bands, RCCL "
                         "all-gather, un-permute on rank 0 (strong scaling, single-frame latency)")
    ap.add_argument("--views", type=int, default=None,
                    help="frames per step (default 16; 1 with --partition bands): a turntable batch of this many "
                         "views of the scene rendered in ONE launch (rt_render_views_device; the drain tail of one "
                         "frame overlaps the next), every frame un-permuted into its own Screen-layout image")
    ap.add_argument("--view-step", type=float, default=None,
                    help="turntable step between views in degrees (default 360 / views)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import rt_amd as R

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # BENCH_DIST_BACKEND=gloo: rehearsal of the N-rank path with several ranks on one GPU (RCCL
        # refuses two ranks on one device); the driver's multi-GPU runs use RCCL ("nccl")
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if local >= torch.cuda.device_count():  # rehearsal: more ranks than GPUs share the visible ones
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    scene, prm, W, H, desc = R.build_config(args.config)
    if args.views is None:
        args.views = 1 if (args.partition == "bands" and world > 1) else DEFAULT_VIEWS
    F = max(1, args.views)
    if F > 1 and args.partition == "bands" and world > 1:
        sys.exit("--views > 1 renders whole frames per rank; use --partition frames")
    cams = R.turntable_cameras(F, R.aspect_of(W, H), args.view_step) if F > 1 else [R.camera_from_trackball(aspect=R.aspect_of(W, H))]
    t_up = time.perf_counter()
    ctx = R.Context(scene, device=local)
    upload_s = time.perf_counter() - t_up

    # frames: each rank is a band split of one (count = 1) -- a whole frame, un-permuted locally
    bands = args.partition == "bands" and world > 1
    b_rank, b_count = (rank, world) if bands else (0, 1)
    nbands = (H + BAND_ROWS - 1) // BAND_ROWS
    max_local = (nbands + b_count - 1) // b_count
    view_elems = max_local * BAND_ROWS * W * 3
    local_buf = torch.zeros(F * view_elems, dtype=torch.float32, device=dev)
    gathered = torch.zeros(world * local_buf.numel(), dtype=torch.float32, device=dev) if bands else local_buf
    image = torch.zeros(F * W * H * 3, dtype=torch.float32, device=dev)

    # one explicit stream for render, gather and un-permute (torch's default stream is the null
    # stream, which would let the un-permute of step k overlap the render of step k+1)
    bstream = torch.cuda.Stream(dev)

    def step():
        with torch.cuda.stream(bstream):
            return _step(bstream.cuda_stream)

    def _step(stream):
        if F > 1:
            st = ctx.render_views_device(cams, prm, W, H, BAND_ROWS, 0, 1, local_buf.data_ptr(), stream)
        else:
            st = ctx.render_device(cams[0], prm, W, H, BAND_ROWS, b_rank, b_count, local_buf.data_ptr(), stream)
        if bands:
            dist.all_gather_into_tensor(gathered, local_buf)
        if rank == 0 or not bands:
            for v in range(F):
                R.check(R.lib().rt_unpermute_bands_device(
                    W, H, BAND_ROWS, b_count, R.C.c_void_p(gathered.data_ptr() + 4 * v * view_elems),
                    R.C.c_void_p(image.data_ptr() + 4 * v * W * H * 3), R.C.c_void_p(stream)))
        return st

    # counting pass (same kernel, COUNT=true) for the algorithmic-byte roofline numerator
    R.set_counting(True)
    cst = step()
    R.set_counting(False)
    for _ in range(args.warmup):
        step()

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    rays = 0
    kms = []
    for _ in range(args.steps):
        st = step()
        rays += st.rays
        kms.append(st.kernel_ms)
    barrier()
    elapsed = time.perf_counter() - t0

    # single-frame latency beside the batch: the default view alone, one launch per frame
    single = None
    if F > 1 and not args.no_single_frame:
        one = ctx.render_device(cams[0], prm, W, H, BAND_ROWS, 0, 1, local_buf.data_ptr(), None)
        n1 = max(5, args.steps)
        barrier()
        t1 = time.perf_counter()
        r1, k1 = 0, []
        for _ in range(n1):
            one = ctx.render_device(cams[0], prm, W, H, BAND_ROWS, 0, 1, local_buf.data_ptr(), None)
            r1 += one.rays
            k1.append(one.kernel_ms)
        barrier()
        e1 = time.perf_counter() - t1
        single = {"ms_per_frame": e1 / n1 * 1e3, "kernel_ms": float(np.mean(k1)), "rays_per_frame": int(one.rays),
                  "Mrays_per_s_per_gpu": r1 / e1 / 1e6, "frames": n1}

    t = torch.tensor([elapsed, float(rays), float(np.mean(kms)), float(cst.node_visits), float(cst.tri_tests),
                      float(cst.hits), float(cst.rays)], dtype=torch.float64, device=dev)
    if world > 1:
        allv = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(allv, t)
        allv = torch.stack(allv).cpu().numpy()
    else:
        allv = t.cpu().numpy()[None, :]
    max_elapsed = float(allv[:, 0].max())
    total_rays = float(allv[:, 1].sum())

    if rank == 0:
        # roofline of the dominant kernel (render_kernel) on rank 0's launches
        pixels0 = int(((nbands - b_rank + b_count - 1) // b_count) * BAND_ROWS * W)
        bytes0 = algorithmic_bytes(cst, F * min(pixels0, W * H))
        avg_ms = float(np.mean(kms))
        achieved = bytes0 / (avg_ms * 1e-3) / 1e9
        kname = kernel_name(ctx.info()["tri_records"])
        pmc = load_pmc(args.config if F == 1 else f"{args.config}/v{F}", kname)
        line = {
            "metric": METRIC,
            "value": total_rays / max_elapsed / 1e6,
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if bands else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 800k-triangle torus-knot stand-in for the missing data/dragon.obj)",
            "config": {"workload": f"{args.config}: {desc}" + (f"; {F} turntable views per step (one launch)"
                                                                  if F > 1 else ""),
                       "resolution": f"{W}x{H}", "frames_per_step": F, "ms_per_frame": max_elapsed / args.steps / F * 1e3,
                       "rays_per_frame": int(total_rays / args.steps / (1 if bands else world) / F),
                       "band_rows": BAND_ROWS,
                       "partition": (f"one frame, {world}-GPU band split" if bands else
                                     f"{world} GPU(s), {F} whole frame(s) per GPU per step"),
                       "scene_upload_s": round(upload_s, 3)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (float(pmc) if pmc is not None else None),
                         "kernel": kname, "kernel_avg_ms": avg_ms,
                         "algorithmic_bytes_per_launch": int(bytes0)},
        }
        if single is not None:
            line["single_frame"] = single
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(args.config, budget_s=args.cpu_budget)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
