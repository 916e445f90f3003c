"""bench.py -- Mrays/s of the MI355X ray tracer on BASELINE.json's 1920x1080 workload.

Workload (config.workload): C3 = dragon proxy (800 000 triangles), 1920x1080,
one point light, hard shadows + mirror recursion depth 4 (BASELINE.json configs[2]).  One step
renders a batch of --views full frames (default 64: a turntable of the scene, 5.625 degrees apart) in
ONE launch of the persistent kernel (rt_render_views_image_device), every pixel stored straight into
its frame's Screen::m_textureData image.  Inputs (scene, BVH) are resident in HBM before timing starts.
--config C4 / C5 measure the other BASELINE configs the same way (C5: 3840x2160).

N > 1 (one process per GPU, torch.distributed "nccl" = RCCL for the control plane): the tile split of
north_star.  Every rank renders its interleaved 8-row bands (band b -> rank b mod N) of ALL the step's
views in one launch, storing each pixel straight into rank 0's images (allocated there and opened by the
other ranks through an IPC handle: the pixel stores cross xGMI while the frame renders, so there is no
gather step after it -- --exchange ipc, the default).  --exchange gather keeps the previous scheme
(band buffers, RCCL gather to rank 0, one un-permute launch there) and is also the fallback when the
IPC mapping fails.  Per-step work is fixed as N grows ("scaling": "strong"), so N = 1 is exactly the
BENCH workload.  --partition frames instead gives each rank its own turntable views (no collective).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config C3] [--views V] [--no-cpu-baseline]
                    [--exchange ipc|gather] [--cpu-pixels P] [--dump-images PATH]

Prints ONE JSON line on rank 0.  `value` = rays (intersect() calls) of the step / max-rank time.
"""
import argparse
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))

import numpy as np  # noqa: E402

METRIC = "Mrays/s (primary+shadow+secondary) at 1920×1080; fraction of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMD-32 units x 2.4 GHz / 2 cycles per wave64 VALU instruction
# (MI355X_MICROARCH.md: "issues each VALU instruction over 2 cycles (32 lanes/cycle x 2)"; one wave alone
# on its SIMD needs 4, so the peak takes >= 2 waves interleaving their VALU)
VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 2
# the SQ counters of the issue / latency picture, one rocprofv3 pass (<= 8 SQ counters per pass)
SQ_PASS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
           "SQ_BUSY_CYCLES")
# the L2 hit rate of the same launches (2 TCC counters, a pass of its own: FETCH_SIZE already takes 3 of the 4)
L2_PASS = ("TCC_HIT_sum", "TCC_MISS_sum")
# cache-served gather rates chip-wide (MI355X_MICROARCH.md "Indexed rows: gather into LDS"): rows served by an XCD's
# L2 16.8-18.8 TB/s, uniformly random rows of a 38 MB table (the Infinity Cache) 8.6 TB/s
L2_GATHER_TBS = 17.8
IC_GATHER_TBS = 8.6
# BASELINE.md's full CPU sample (4 096 pixels of the seed-12345 permutation for C3-C5, whole frames for C1 / C2),
# timed by tools/cpu_baseline.py on the GPU box's host; the bench line's own leg is a bounded prefix of it
CPU_FULL = os.path.join("profiles", "r06", "cpu_baseline_full.json")
BAND_ROWS = 8
DEFAULT_VIEWS = 64  # frames per step: a 64-view turntable (5.625 deg apart) of the C3 scene in one launch
# frames per step of the other configs (a step of a few hundred ms at most): C4's 64-sample soft shadows
# take ~10 ms per frame; a C5 4K frame (3 x 64 plane-light samples, glass to depth 8: ~1e9 rays) fills the GPU
# on its own, and batching its views measured slower per ray (2 900 vs 2 556 Mrays/s for 8 views, r02)
CONFIG_VIEWS = {"C1": 64, "C2": 64, "C3": DEFAULT_VIEWS, "C4": 16, "C5": 1}


def algorithmic_bytes(st, pixels):
    """one node record per node visit (128 B: the quantised BVH8 the kernel walks),
    64 B per triangle record, 68 B per shaded hit (3 normals + material), 12 B per pixel written."""
    return int(st.node_bytes or 128) * st.node_visits + 64 * st.tri_tests + 68 * st.hits + 12 * pixels


def lib_sha():
    import rt_amd as R

    with open(R.LIB_PATH, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_threads():
    """The host cores this process may use: OMP_NUM_THREADS where set (the GPU box sets its CPU
    share there; os.cpu_count() reports the whole machine), else os.cpu_count()."""
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(os.cpu_count() or 1, n if n > 0 else (os.cpu_count() or 1)))


def cpu_baseline(config, budget_s=12.0, seed=12345, max_pixels=None):
    """The reference algorithm (oracle/ref_cpu.cpp, g++ -O2 -fopenmp) timed on the host: brute-force
    primary/secondary rays (useBVH=false, the reference default, src/main.cpp:60) and the reference's
    own depth-4 BVH (useBVH=true), each single-threaded and on every host core, on the first pixels
    of BASELINE.md's seed-12345 permutation of the frame (rays counted exactly).  Each leg stops at
    budget_s / 4 seconds or max_pixels pixels (BASELINE.md's sample: 4 096 for C3-C5, the whole frame for
    C1/C2; tools/cpu_baseline.py runs those in full)."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    scene, prm, W, H, _ = R.build_config(config)
    orc = O.Oracle(scene)
    order = np.random.default_rng(seed).permutation(W * H)
    if max_pixels:
        order = order[:max_pixels]
    allc = host_threads()
    legs = {}
    for bvh in (0, 1):
        p = R.rt_params.from_buffer_copy(prm)
        p.use_bvh = bvh
        for threads in (1, allc):
            O.set_threads(threads)
            rays, npx = 0, 0
            chunk = 4 * threads
            t0 = time.perf_counter()
            while time.perf_counter() - t0 < budget_s / 4 and npx < len(order):
                sel = order[npx:npx + chunk]
                xy = np.stack([sel % W, sel // W], axis=1)
                _, r = orc.render_pixels(p, W, H, xy)
                rays += int(r.sum())
                npx += len(sel)
            dt = time.perf_counter() - t0
            key = f"{'1core' if threads == 1 else 'allcore'}_bvh{bvh}"
            legs[key] = {"value": rays / dt / 1e6, "cores": threads, "pixels": npx, "rays": rays,
                         "seconds": round(dt, 2)}
    base = legs["1core_bvh0"]
    whole = all(v["pixels"] == W * H for v in legs.values())
    full = None
    try:  # BASELINE.md's whole sample, timed once in full (tools/cpu_baseline.py) on the GPU box's host
        with open(os.path.join(REPO, CPU_FULL)) as f:
            for c in json.load(f)["configs"]:
                if c["config"] == config:
                    full = {"file": CPU_FULL, "sample": c["sample"],
                            "legs": {k: {"Mrays_per_s": v["Mrays_per_s"], "threads": v["threads"], "pixels": v["pixels"],
                                         "seconds": v["seconds"]} for k, v in c["legs"].items()}}
    except (OSError, ValueError, KeyError):
        pass
    if whole:
        return {"value": base["value"], "unit": "Mrays/s", "cores": 1, "kind": "port",
                "sample": f"BASELINE.md's sample for {config}: the whole {W}x{H} frame, {base['rays']} rays in "
                          f"{base['seconds']} s single-threaded, useBVH=false (reference default); legs: 1 / {allc} "
                          f"threads x useBVH false / true; host CPU: {_cpu_model()}",
                "legs": legs}
    return {"value": base["value"], "unit": "Mrays/s", "cores": 1, "kind": "port",
            "sample": f"bounded prefix of BASELINE.md's sample (the first pixels of the seed-{seed} permutation of "
                      f"{config} {W}x{H}): {base['pixels']} pixels, {base['rays']} rays in {base['seconds']} s "
                      f"single-threaded, useBVH=false (reference default); legs: 1 / {allc} threads x useBVH false / "
                      f"true; host CPU: {_cpu_model()}; the whole sample (4 096 pixels for C3-C5) timed in full: "
                      f"full_sample ({CPU_FULL})",
            "legs": legs, "full_sample": full}


def pmc_key(config, views):
    """The config key of a PMC summary (tools/pmc_summary.py's CONFIG argument): e.g. C3v64."""
    return f"{config}v{views}"


def measure_pmc(config, views, kernel, timeout_s=150):
    """HBM bytes and VALU instructions per render launch measured now: three rocprofv3 --pmc passes
    (FETCH_SIZE, WRITE_SIZE -- together they exceed the 4 TCC counters one pass can hold -- and
    SQ_INSTS_VALU) over tools/prof_target.py, which makes the same launches this bench times (config,
    views, library); per MI355X_MICROARCH.md's HBM section FETCH_SIZE and WRITE_SIZE are KB and gfx950's
    FETCH_SIZE tallies 128-B requests at 64 B, so bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
    Returns (bytes or None, provenance, {counter: median per launch})."""
    import shutil
    import subprocess
    import tempfile

    sys.path.insert(0, os.path.join(REPO, "tools"))
    import pmc_summary

    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found", {}
    med = {}
    with tempfile.TemporaryDirectory(prefix="bench_pmc_") as tmp:
        for group in (("FETCH_SIZE",), ("WRITE_SIZE",), SQ_PASS, L2_PASS):
            out = os.path.join(tmp, group[0])
            cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", *group, "--kernel-trace", "--output-format",
                   "csv", "-d", out, "-o", "run", "--", sys.executable, os.path.join(REPO, "tools", "prof_target.py"),
                   config, "2", str(views)]
            r = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO)
            if r.returncode != 0:
                return None, f"rocprofv3 --pmc {' '.join(group)} failed (rc {r.returncode}): {(r.stderr or r.stdout)[-300:]}", med
            kname, m = pmc_summary.collect(out)
            if any(c not in m for c in group) or not kname or kernel not in kname:
                return None, f"rocprofv3 --pmc {' '.join(group)}: no counter rows for {kernel}", med
            med.update({c: m[c] for c in group})
    hbm = (2.0 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024.0
    return hbm, (f"measured in this run: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/prof_target.py "
                 f"{config} {views} views (the same kernel and library), median per launch; FETCH_SIZE "
                 f"{med['FETCH_SIZE']:.0f} KB (x2, gfx950 64-B tally of 128-B requests), WRITE_SIZE "
                 f"{med['WRITE_SIZE']:.0f} KB"), med


def load_pmc(config, kernel, sha, path=None):
    """HBM bytes per render launch from the committed rocprofv3 --pmc summary
    (profiles/pmc_latest.json, written by tools/pmc_summary.py --latest) -- used only when it was
    measured on this exact library build (sha) and kernel; returns (bytes or None, provenance)."""
    p = path or os.path.join(REPO, "profiles", "pmc_latest.json")
    try:
        with open(p) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no profiles/pmc_latest.json"
    if d.get("config") != config or kernel not in (d.get("kernel") or ""):
        return None, f"profiles/pmc_latest.json is for {d.get('config')} / {d.get('kernel')}"
    if d.get("lib_sha") != sha:
        return None, f"profiles/pmc_latest.json was measured on library {d.get('lib_sha')}, this is {sha}"
    return d.get("hbm_bytes_per_launch"), (f"profiles/pmc_latest.json: rocprofv3 --pmc of this library "
                                           f"({sha}), {d.get('note', '')}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=16.0, help="seconds of CPU baseline work (4 legs)")
    ap.add_argument("--no-single-frame", action="store_true",
                    help="skip the single-frame latency record (profiling runs: one kernel shape only)")
    ap.add_argument("--partition", choices=("bands", "frames"), default="bands",
                    help="N>1: bands = every view of the step split into interleaved 8-row bands over the ranks, "
                         "the pixels exchanged into rank 0's images as --exchange says (north_star's tile split, strong "
                         "scaling); frames = every rank renders its own turntable views (weak scaling, no collective "
                         "on the data path)")
    ap.add_argument("--views", type=int, default=None,
                    help="frames per step, rendered in ONE launch (default per config: C3 64, C4 16, C5 2)")
    ap.add_argument("--view-step", type=float, default=None,
                    help="turntable step between views in degrees (default 360 / views)")
    ap.add_argument("--exchange", choices=("ipc", "gather", "none"), default="ipc",
                    help="N>1 bands: ipc = every rank stores its pixels straight into rank 0's images (IPC-mapped, "
                         "no gather step); gather = band buffers + RCCL gather + un-permute on rank 0; none = the "
                         "control leg: every rank stores its bands into its OWN images (the same render work with no "
                         "exchange, so a scaling run can separate the exchange's cost)")
    ap.add_argument("--cpu-pixels", type=int, default=0,
                    help="CPU baseline: stop each leg at this many pixels as well as at --cpu-budget (0: budget only)")
    ap.add_argument("--resolution", default=None, help="WxH override (tests; the BENCH line uses the config's)")
    ap.add_argument("--dragon-uv", default=None, help="UxV dragon-proxy tessellation override (tests)")
    ap.add_argument("--dump-images", default=None, help="rank 0 saves the last step's images (.npy; tests)")
    ap.add_argument("--no-pmc", action="store_true",
                    help="skip the two rocprofv3 --pmc passes that measure roofline.traffic (N = 1)")
    args = ap.parse_args()
    if args.views is None:
        args.views = CONFIG_VIEWS.get(args.config, DEFAULT_VIEWS)

    import torch
    import torch.distributed as dist
    import rt_amd as R

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # BENCH_DIST_BACKEND=gloo: rehearsal of the N-rank path with several ranks on one GPU or on the
        # CPU (RCCL refuses two ranks on one device); the driver's multi-GPU runs use RCCL ("nccl")
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    if local >= torch.cuda.device_count():  # rehearsal: more ranks than GPUs share the visible ones
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    # the library measured must be the one built from this tree's sources (raises otherwise)
    prov = R.provenance()
    uv = tuple(int(x) for x in args.dragon_uv.split("x")) if args.dragon_uv else None
    scene, prm, W, H, desc = R.build_config(args.config, dragon_uv=uv)
    if args.resolution:
        W, H = (int(x) for x in args.resolution.split("x"))
    F = max(1, args.views)
    bands = args.partition == "bands"
    b_rank, b_count = (rank, world) if bands else (0, 1)
    if bands:
        eulers = R.turntable_eulers(F, args.view_step)
    else:  # every rank renders different frames of one turntable
        eulers = R.turntable_eulers(F * world, args.view_step)[rank * F:(rank + 1) * F]
    cams = [R.camera_from_trackball(euler=e, aspect=R.aspect_of(W, H)) for e in eulers]
    # scene upload (rt_create: GPU build of the acceleration structures + uploads); the first context
    # of a process also loads the library's code objects, so the steady-state figure is a second build
    t_up = time.perf_counter()
    ctx = R.Context(scene, device=local)
    upload_cold_s = time.perf_counter() - t_up
    ctx.close()
    t_up = time.perf_counter()
    ctx = R.Context(scene, device=local)
    upload_s = time.perf_counter() - t_up
    build_info = ctx.build_info()

    img_elems = F * W * H * 3
    exchange = "local" if (world == 1 or not bands) else args.exchange
    # (images of 2 GiB or more: rt_ipc_alloc refuses them -- this ROCm's hipIpcOpenMemHandle never returns for such
    # a buffer, tools/ipc_probe.py, DESIGN.md section 7 -- and the ranks fall back to the gather scheme below)
    ipc = None
    if exchange == "ipc":
        # rank 0's images, opened by every other rank: the ranks' kernels store their pixels into them.  Every
        # rank takes part in the broadcast whatever rank 0's allocation did (None: no buffer), so a failure on
        # any rank falls back to the gather scheme instead of leaving the ranks in mismatched collectives.
        ok, handle = 1, None
        if rank == 0:
            try:
                if os.environ.get("BENCH_IPC_FAIL_RANK0"):  # test hook: rank 0's export fails
                    raise R.RtError("rt_ipc_alloc: forced failure (BENCH_IPC_FAIL_RANK0)")
                ipc = R.IpcBuffer(local, nbytes=img_elems * 4)
                handle = ipc.handle
            except R.RtError as e:
                print(f"rank 0: IPC export failed ({e}); falling back to --exchange gather", file=sys.stderr)
                ok = 0
        obj = [handle]
        dist.broadcast_object_list(obj, src=0)
        if rank != 0:
            if obj[0] is None:
                ok = 0
            else:
                try:
                    ipc = R.IpcBuffer(local, handle=obj[0])
                except R.RtError as e:  # no IPC on this node: the gather scheme
                    print(f"rank {rank}: IPC mapping failed ({e}); falling back to --exchange gather", file=sys.stderr)
                    ok = 0
        flag = torch.tensor([ok], dtype=torch.int32, device=dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if not int(flag.item()):
            if ipc is not None:
                ipc.close()
            ipc = None
            exchange = "gather"
    # (exchange "none": every rank's own images, the control leg; "local": N = 1 or frames)
    images = None if exchange == "ipc" else torch.zeros(img_elems, dtype=torch.float32, device=dev)
    img_ptr = ipc.ptr if exchange == "ipc" else images.data_ptr()
    nbands = (H + BAND_ROWS - 1) // BAND_ROWS
    max_local = (nbands + b_count - 1) // b_count
    if exchange == "gather":
        view_elems = max_local * BAND_ROWS * W * 3
        local_buf = torch.zeros(F * view_elems, dtype=torch.float32, device=dev)
        # RCCL: gather to rank 0; the gloo rehearsal (BENCH_DIST_BACKEND=gloo, device tensors) all-gathers instead
        to_root = dist.get_backend() == "nccl"
        gathered = (torch.zeros(b_count * local_buf.numel(), dtype=torch.float32, device=dev)
                    if rank == 0 or not to_root else None)
    torch.cuda.synchronize(dev)  # the fills above ran on torch's default stream; the renders use bstream

    # one explicit stream for the step's work (torch's default stream is the null stream)
    bstream = torch.cuda.Stream(dev)

    def step(cams_=cams):
        with torch.cuda.stream(bstream):
            if exchange != "gather":  # each pixel straight into its image (rank 0's, IPC-mapped, for N > 1)
                return ctx.render_views_image_device(cams_, prm, W, H, img_ptr, bstream.cuda_stream, band_rank=b_rank,
                                                     band_count=b_count)
            st = ctx.render_views_device(cams_, prm, W, H, BAND_ROWS, b_rank, b_count, local_buf.data_ptr(),
                                         bstream.cuda_stream)
            if to_root:  # to rank 0 only: each rank's bands cross one xGMI link, all at once
                dist.gather(local_buf, gather_list=list(gathered.chunk(b_count)) if rank == 0 else None, dst=0)
            else:
                dist.all_gather_into_tensor(gathered, local_buf)
            if rank == 0:
                R.check(R.lib().rt_unpermute_views_device(W, H, BAND_ROWS, b_count, len(cams_),
                                                          R.C.c_void_p(gathered.data_ptr()),
                                                          R.C.c_void_p(images.data_ptr()),
                                                          R.C.c_void_p(bstream.cuda_stream)), "unpermute")
        return st

    # counting pass (same kernel, COUNT=true) for the algorithmic-byte roofline numerator and the
    # count of hits in the reference's undefined-barycentrics regime
    R.set_counting(True)
    cst = step()
    R.set_counting(False)
    # lane use of the traversal (counting build): lane node visits / (64 x wave node steps), same for records
    cdbg = [int(x) for x in ctx.debug_counters()[:28]]
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
    st = None
    for _ in range(args.steps):
        st = step()
        rays += st.rays
        kms.append(st.kernel_ms)
    barrier()
    elapsed = time.perf_counter() - t0

    # single-frame latency beside the batch: the default view alone (this rank's bands), one launch
    single = None
    if F > 1 and not args.no_single_frame:
        one_cam = [R.camera_from_trackball(aspect=R.aspect_of(W, H))]

        def frame():
            if exchange != "gather":  # into view 0 of the images (rank 0's for N > 1)
                return step(one_cam)
            # gather scheme: the rank's bands of the frame alone (per-GPU latency, no gather)
            return ctx.render_device(one_cam[0], prm, W, H, BAND_ROWS, b_rank, b_count, local_buf.data_ptr(), None)

        one = frame()
        n1 = max(5, args.steps)
        barrier()
        t1 = time.perf_counter()
        r1, k1 = 0, []
        for _ in range(n1):
            one = frame()
            r1 += one.rays
            k1.append(one.kernel_ms)
        barrier()
        e1 = time.perf_counter() - t1
        single = {"ms_per_frame": e1 / n1 * 1e3, "kernel_ms": float(np.mean(k1)), "rays_per_frame": int(one.rays),
                  "Mrays_per_s_per_gpu": r1 / e1 / 1e6, "frames": n1, "kernel": one.kernel_name}
        step()  # the last step's images again (--dump-images)
        barrier()

    if args.dump_images and rank == 0:
        if exchange == "ipc":
            out = R.device_to_host(img_ptr, img_elems)
        else:
            out = images.cpu().numpy()
        np.save(args.dump_images, out.reshape(F, -1))

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
        # roofline of the dominant kernel (the persistent render kernel) on rank 0's launches
        pixels0 = int(max_local * BAND_ROWS * W) if b_count > 1 else W * H
        bytes0 = algorithmic_bytes(cst, F * min(pixels0, W * H))
        avg_ms = float(np.mean(kms))
        achieved = bytes0 / (avg_ms * 1e-3) / 1e9
        kname = st.kernel_name
        sha = lib_sha()
        pmc, pmc_src, pmc_med = None, "not measured (--no-pmc or N > 1)", {}
        if world == 1 and not args.no_pmc and not args.resolution and not args.dragon_uv:
            pmc, pmc_src, pmc_med = measure_pmc(args.config, F, kname)
        if pmc is None and world == 1:  # the committed summary (one GPU's whole launch), same library build only
            pmc_c, src_c = load_pmc(pmc_key(args.config, F), kname, sha)
            if pmc_c is not None:
                pmc, pmc_src = pmc_c, src_c
            else:
                pmc_src += f"; {src_c}"
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
            "config": {"workload": f"{args.config}: {desc}; {F} turntable views per step (one launch)",
                       "resolution": f"{W}x{H}", "frames_per_step": F,
                       "ms_per_frame": max_elapsed / args.steps / F * 1e3,
                       "rays_per_frame": int(total_rays / args.steps / (1 if bands else world) / F),
                       "band_rows": BAND_ROWS,
                       "partition": (f"{world}-GPU tile split: interleaved 8-row bands of every view, "
                                     + ("each rank's pixels stored straight into rank 0's images (IPC-mapped, "
                                        "stores over xGMI while rendering; no gather step)" if exchange == "ipc" else
                                        "NO exchange (control leg: each rank stores its bands into its own images)"
                                        if exchange == "none" else
                                        "RCCL gather to rank 0 + un-permute" if to_root else
                                        f"{dist.get_backend()} all-gather + un-permute")
                                     if bands and world > 1 else
                                     f"{world} GPU(s), {F} whole frame(s) per GPU per step, pixels stored in "
                                     "their images (setPixel layout)"),
                       "scene_upload_s": round(upload_s, 4),
                       "scene_upload_first_s": round(upload_cold_s, 3),
                       "scene_build": "GPU (rt_build.hip)" if build_info["gpu"] else "host (bvh_build.cpp)",
                       "ub_regime_hits": {"hits": int(cst.hits), "ub": int(cst.ub_hits),
                                          "share": (cst.ub_hits / cst.hits) if cst.hits else 0.0,
                                          "note": "shaded triangle hits where the reference's barycentricCoordinates "
                                                  "returns false (src/ray_tracing.cpp:281-295): rank 0's bands, "
                                                  "counting pass"}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": (float(pmc) if pmc is not None else None), "traffic_source": pmc_src,
                         "kernel": kname, "lib_sha": sha, "source_hash": prov["library_source_hash"],
                         "kernel_avg_ms": avg_ms,
                         "algorithmic_bytes_per_launch": int(bytes0)},
        }
        lane_use = {"node_steps": cdbg[1] / max(1, 64 * cdbg[4]), "record_steps": cdbg[2] / max(1, 64 * cdbg[5]),
                    "source": "counting pass of the same kernel (rt_debug_counters): lane visits / (64 x wave steps)"}
        if "SQ_INSTS_VALU" in pmc_med:
            # the VALU issue roofline beside SURVEY.md §8d's algorithmic-byte one (achieved / peak / frac above stay
            # the HBM figures of the contract).  The kernels are branchy scalar FP32 whose bytes come mostly from L2 /
            # MALL, so neither peak binds: "limiter" names what the wave-cycle counters show (waiting on memory vs
            # issuing) beside the issue fraction against the SIMD-32 peak and the lanes' use of each traversal step
            vi = float(pmc_med["SQ_INSTS_VALU"])
            ia = vi / (avg_ms * 1e-3)
            line["roofline"]["issue"] = {
                "achieved": ia, "peak": VALU_PEAK_WAVE_INSTR_S, "unit": "wave-instructions/s",
                "frac": ia / VALU_PEAK_WAVE_INSTR_S, "valu_insts_per_launch": vi,
                "valu_insts_per_ray": vi / max(1.0, float(cst.rays)),
                "salu_per_valu": float(pmc_med.get("SQ_INSTS_SALU", 0.0)) / max(1.0, vi),
                "source": "rocprofv3 --pmc SQ_INSTS_VALU (median per launch, same run) / kernel_avg_ms; peak = 256 CUs "
                          "x 4 SIMD-32 x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md)"}
            wc = float(pmc_med.get("SQ_WAVE_CYCLES", 0.0))
            split = ({k: float(pmc_med[k]) / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
                      if k in pmc_med} if wc > 0 else {})
            issue_frac = ia / VALU_PEAK_WAVE_INSTR_S
            waiting = split.get("SQ_WAIT_ANY", 0.0)
            kind = ("memory latency + lane divergence" if waiting > split.get("SQ_ACTIVE_INST_ANY", 1.0)
                    and issue_frac < 0.7 else "valu-issue" if issue_frac >= 0.7 else "mixed issue / latency")
            line["roofline"]["limiter"] = {
                "kind": kind, "issue_frac": issue_frac, "wave_cycles": split, "lane_use": lane_use,
                "note": "share of wave cycles issuing (SQ_ACTIVE_INST_ANY) / waiting on memory (SQ_WAIT_ANY) / waiting "
                        "on a dependency (SQ_WAIT_INST_ANY), same rocprofv3 pass; the HBM fraction above is "
                        "algorithmic bytes (SURVEY.md 8d), most of them served by L2 / MALL (traffic = DRAM bytes)"}
        else:
            line["roofline"]["limiter"] = {"lane_use": lane_use}
        if "TCC_HIT_sum" in pmc_med:
            # beside the HBM fraction (SURVEY.md 8d's algorithmic bytes over the HBM peak): the rate the caches serve
            # such gathers at, weighted by this run's L2 hit rate -- the time-weighted blend of the guide's L2 and
            # Infinity-Cache gather rates.  The guide measured whole 1 152-B rows; the kernel gathers 16-B pieces per
            # lane, so this is an approximate ceiling
            hits_, miss_ = float(pmc_med["TCC_HIT_sum"]), float(pmc_med["TCC_MISS_sum"])
            h = hits_ / max(1.0, hits_ + miss_)
            ceil_tbs = 1.0 / (h / L2_GATHER_TBS + (1.0 - h) / IC_GATHER_TBS)
            line["roofline"]["cache_ceiling"] = {
                "l2_hit": h, "l2_gather_TBs": L2_GATHER_TBS, "ic_gather_TBs": IC_GATHER_TBS, "ceiling_GBs": ceil_tbs * 1e3,
                "frac": achieved / (ceil_tbs * 1e3),
                "source": "rocprofv3 --pmc TCC_HIT_sum / TCC_MISS_sum (median per launch, same run); rates from "
                          "MI355X_MICROARCH.md 'Indexed rows: gather into LDS' (L2 16.8-18.8 TB/s, Infinity Cache 8.6 "
                          "TB/s; whole-row gathers, so approximate for 16-B per-lane pieces)"}
        # the ray mix of the counting pass (rank 0's launch): camera rays are one per pixel and sample; the kernels
        # count cansee segments / light samples and the camera rays that hit nothing (rt_debug_counters [26], [27])
        samples = 4 if prm.anti_aliasing else (int(prm.sample_size) if prm.multiple_rays else 1)
        cam = F * min(pixels0, W * H) * samples
        shad, cmiss = cdbg[26], cdbg[27]
        crays = int(cst.rays)
        line["config"]["ray_mix"] = {
            "rays": crays, "camera": cam, "camera_no_hit": cmiss, "shadow_segments": shad,
            "secondary": crays - cam - shad, "shaded_hits": int(cst.hits),
            "ns_per_shaded_hit": avg_ms * 1e6 / max(1, int(cst.hits)),
            "ns_per_ray": avg_ms * 1e6 / max(1, crays),
            "note": "one launch of the step (counting pass, rank 0): camera = pixels x samples; shadow_segments = cansee "
                    "segments and light samples; secondary = mirror / reflected / refracted rays; ns_per_shaded_hit = "
                    "kernel time / shaded hits (a speed-up of background camera rays alone does not move it)"}
        if single is not None:
            line["single_frame"] = single
        if world == 1 and not args.no_cpu_baseline:
            # C1 / C2: BASELINE.md times the whole frame (C2 ~30 s over the four legs on the box's host); C3-C5 a
            # bounded prefix of the 4 096-pixel sample (the whole sample: tools/cpu_baseline.py)
            whole = args.config in ("C1", "C2") and not args.cpu_pixels
            line["cpu_baseline"] = cpu_baseline(args.config, budget_s=480.0 if whole else args.cpu_budget,
                                                max_pixels=args.cpu_pixels or None)
        print(json.dumps(line), flush=True)
    ctx.close()  # explicitly: no HIP teardown left to interpreter exit
    if ipc is not None and not ipc.owner:  # the importers unmap rank 0's images before rank 0 frees them
        ipc.close()
    if world > 1:
        dist.barrier()
    if ipc is not None:
        ipc.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
