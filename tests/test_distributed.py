"""World-size-2 gloo rehearsal of the multi-GPU path (bench.py): each rank renders its interleaved
8-row bands, the padded band buffers are all-gathered and rank 0 un-permutes them.  The bands are
rendered here by the CPU oracle (no GPU in this container); the GPU test
tests/test_gpu_parity.py::test_band_split_bit_identical runs the same layout through the HIP kernel."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, W, H, band_rows, out_path):
    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    O.set_threads(1)
    scene, prm, _, _, _ = R.build_config("C2")
    orc = O.Oracle(scene)
    rows = R.band_rows_of(H, band_rows, rank, world)
    xy = np.array([(x, y) for y in rows for x in range(W)], np.int32)
    rgb, rays = orc.render_pixels(prm, W, H, xy)
    local = np.zeros(R.local_band_elems(W, H, band_rows, world), np.float32)
    local[:rgb.size] = rgb.reshape(-1)
    t = torch.from_numpy(local)
    gathered = torch.zeros(world * t.numel(), dtype=torch.float32)
    dist.all_gather_into_tensor(gathered, t)
    total = torch.tensor([float(rays.sum())], dtype=torch.float64)
    dist.all_reduce(total)
    if rank == 0:
        img = R.unpermute_host(gathered.numpy(), W, H, band_rows, world)
        np.savez(out_path, img=img, rays=total.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,band_rows", [(2, 24, 20, 8), (2, 17, 9, 4), (3, 16, 33, 8)])
def test_band_split_gather_matches_single_render(tmp_path, world, W, H, band_rows):
    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    out = str(tmp_path / "img.npz")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, band_rows, out), nprocs=world, join=True,
                       start_method="spawn")
    z = np.load(out)
    scene, prm, _, _, _ = R.build_config("C2")
    ref, rays = O.Oracle(scene).render(prm, W, H)
    assert z["img"].tobytes() == ref.tobytes()
    assert int(z["rays"][0]) == rays


def test_band_rows_cover_image_once():
    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    import rt_amd as R

    for H, br, n in [(1080, 8, 8), (1080, 8, 3), (2160, 8, 7), (5, 8, 2)]:
        rows = [r for k in range(n) for r in R.band_rows_of(H, br, k, n)]
        assert sorted(rows) == list(range(H))


def _expand_scenes(cache, q):
    import os
    import sys

    os.environ["RT_SCENE_CACHE"] = cache
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracer-group27_amd"))
    try:
        import rt_amd

        rt_amd.data_dir()
        q.put("ok")
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


def test_ranks_expand_scene_cache_concurrently(tmp_path):
    """Every rank of a node expands the gzipped reference scenes into the same cache directory at
    start-up (bench.py on N GPUs): concurrent expansion must not collide.  Checked once every
    process has joined: each expected file is present and complete, and no temporary is left."""
    import gzip
    import multiprocessing as mp

    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    import rt_amd as R

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    cache = str(tmp_path / "scenes")
    ps = [ctx.Process(target=_expand_scenes, args=(cache, q)) for _ in range(6)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert res == ["ok"] * len(ps), res
    expected = sorted(f[:-3] for f in os.listdir(R.SCENE_DIR) if f.endswith(".gz"))
    present = sorted(os.listdir(cache))
    assert present == expected  # nothing missing, no *.tmp left behind
    for f in expected:
        with gzip.open(os.path.join(R.SCENE_DIR, f + ".gz"), "rb") as g, open(os.path.join(cache, f), "rb") as h:
            assert g.read() == h.read(), f


def _views_worker(rank, world, port, W, H, band_rows, n_views, out_path, to_root):
    """bench.py's N-rank step, with the oracle in place of the GPU: this rank's interleaved bands of
    every view of the turntable batch, packed as rt_render_views_device packs them, gathered to rank 0
    (to_root: dist.gather into chunks of one buffer, bench.py's RCCL path) or all-gathered (its gloo
    rehearsal), un-permuted on rank 0 (rt_unpermute_views_device's host statement)."""
    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    O.set_threads(1)
    scene, prm, _, _, _ = R.build_config("C2")
    orc = O.Oracle(scene)
    rows = R.band_rows_of(H, band_rows, rank, world)
    xy = np.array([(x, y) for y in rows for x in range(W)], np.int32)
    per_view = R.local_band_elems(W, H, band_rows, world)
    local = np.zeros(n_views * per_view, np.float32)
    rays = 0
    for v, e in enumerate(R.turntable_eulers(n_views)):
        rgb, r = orc.render_pixels(prm, W, H, xy, euler=e)
        local[v * per_view:v * per_view + rgb.size] = rgb.reshape(-1)
        rays += int(r.sum())
    t = torch.from_numpy(local)
    gathered = torch.zeros(world * t.numel(), dtype=torch.float32) if rank == 0 or not to_root else None
    if to_root:
        dist.gather(t, gather_list=list(gathered.chunk(world)) if rank == 0 else None, dst=0)
    else:
        dist.all_gather_into_tensor(gathered, t)
    total = torch.tensor([float(rays)], dtype=torch.float64)
    dist.all_reduce(total)
    if rank == 0:
        imgs = R.unpermute_views_host(gathered.numpy(), W, H, band_rows, world, n_views)
        np.savez(out_path, imgs=imgs, rays=total.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("to_root", [True, False], ids=["gather", "all_gather"])
@pytest.mark.parametrize("world,W,H,n_views", [(2, 20, 19, 3), (3, 16, 33, 2)])
def test_band_split_of_view_batch_matches_single_renders(tmp_path, world, W, H, n_views, to_root):
    """The default N>1 bench layout (north_star's tile split of the benchmarked view batch): every
    gathered view equals the single-process render of that view, ray counts add up."""
    sys.path.insert(0, os.path.join(REPO, "raytracer-group27_amd"))
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O
    import rt_amd as R

    out = str(tmp_path / "views.npz")
    mp.start_processes(_views_worker, args=(world, _free_port(), W, H, 8, n_views, out, to_root), nprocs=world, join=True,
                       start_method="spawn")
    z = np.load(out)
    scene, prm, _, _, _ = R.build_config("C2")
    o = O.Oracle(scene)
    total = 0
    for v, e in enumerate(R.turntable_eulers(n_views)):
        ref, rays = o.render(prm, W, H, euler=e)
        assert z["imgs"][v].tobytes() == ref.tobytes(), v
        total += rays
    assert int(z["rays"][0]) == total
