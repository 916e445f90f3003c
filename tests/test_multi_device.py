"""The tile split behind the C-ABI: rt_create over a device list renders every
frame's interleaved 8-row bands on its replicas, each storing pixels straight into the setPixel layout
on devices[0] -- and the one-process-per-GPU form of the same split (bench.py N > 1: rank 0's images
opened by the other ranks through an IPC handle).

On the one-GPU test box the "devices" are replicas on GPU 0 ({0, 0}, {0, 0, 0}): the same code path as
a multi-GPU node except that the peer stores stay on one device.  Everything must be bit-identical to the
single-device render, and the single-device render must be bit-identical to the band-dense render +
un-permute of rounds 1-2 (the previous layout)."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (config, dragon tessellation, W, H): C3 mirror recursion, C4 spherical-light fans (interleaved jobs
# for single frames, whose job decode depends on the band rank), C5 glass + plane-light fans at depth 8
CASES = [("C3", (200, 80), 200, 123), ("C4", (200, 80), 96, 54), ("C5", None, 96, 54)]


@pytest.fixture(scope="module")
def scenes(R):
    cache = {}

    def get(cfg, uv):
        if (cfg, uv) not in cache:
            scene, prm, _, _, _ = R.build_config(cfg, dragon_uv=uv)
            cache[(cfg, uv)] = (scene, prm, R.Context(scene))
        return cache[(cfg, uv)]

    yield get
    for _, _, ctx in cache.values():
        ctx.close()


def _band_dense(R, ctx, cam, prm, W, H):
    """Rounds 1-2's layout: rt_render_device bands + rt_unpermute_bands_device."""
    import torch

    n = R.local_band_elems(W, H, 8, 1)
    buf = torch.full((n,), -1.0, dtype=torch.float32, device="cuda")
    st = ctx.render_device(cam, prm, W, H, 8, 0, 1, buf.data_ptr(), None)
    img = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    R.check(R.lib().rt_unpermute_bands_device(W, H, 8, 1, ctypes.c_void_p(buf.data_ptr()),
                                              ctypes.c_void_p(img.data_ptr()), None))
    torch.cuda.synchronize()
    return img.cpu().numpy(), st


@pytest.mark.parametrize("cfg,uv,W,H", CASES, ids=[c[0] for c in CASES])
def test_replicas_bit_identical(R, scenes, cfg, uv, W, H):
    scene, prm, ctx1 = scenes(cfg, uv)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    ref, st = ctx1.render(cam, prm, W, H)
    dense, std = _band_dense(R, ctx1, cam, prm, W, H)
    assert ref.tobytes() == dense.tobytes()  # {0}: today's bits in the new (setPixel) layout
    assert st.rays == std.rays
    for devs in ([0, 0], [0, 0, 0]):
        ctx = R.Context(scene, devices=devs)
        try:
            assert ctx.devices == devs
            assert ctx.peer_stores() == [True] * len(devs)
            img, s = ctx.render(cam, prm, W, H)
            assert img.tobytes() == ref.tobytes(), devs
            assert s.rays == st.rays, devs
            # the exchange of devices without peer access: band-dense renders copied to devices[0] and
            # scattered into place there (RT_OPT_PEER_STORES 0 forces it for every extra replica)
            ctx.set_option(R.OPT_PEER_STORES, 0)
            assert ctx.peer_stores() == [True] + [False] * (len(devs) - 1)
            img, s = ctx.render(cam, prm, W, H)
            assert img.tobytes() == ref.tobytes(), (devs, "copy exchange")
            assert s.rays == st.rays, devs
        finally:
            ctx.close()


@pytest.mark.parametrize("cfg,uv,W,H", CASES, ids=[c[0] for c in CASES])
def test_replicas_view_batch_and_rank_split(R, scenes, cfg, uv, W, H):
    """View batches split over replicas; and two 'process ranks' (band_rank 0 / 1 of 2) each splitting
    their bands over a 2-replica context fill one image buffer exactly like one full render."""
    import torch

    scene, prm, ctx1 = scenes(cfg, uv)
    cams = R.turntable_cameras(3, R.aspect_of(W, H))
    ref, st = ctx1.render_views(cams, prm, W, H)
    ctx = R.Context(scene, devices=[0, 0])
    try:
        for peer in (-1, 0):  # peer stores, then the band-copy exchange
            ctx.set_option(R.OPT_PEER_STORES, peer)
            got, s = ctx.render_views(cams, prm, W, H)
            assert got.tobytes() == ref.tobytes(), peer
            assert s.rays == st.rays
            imgs = torch.full((3 * W * H * 3,), -1.0, dtype=torch.float32, device="cuda")
            rays = 0
            for rank in range(2):
                rays += ctx.render_views_image_device(cams, prm, W, H, imgs.data_ptr(), None, band_rank=rank,
                                                      band_count=2).rays
            torch.cuda.synchronize()
            assert imgs.cpu().numpy().reshape(3, -1).tobytes() == ref.tobytes(), peer
            assert rays == st.rays
    finally:
        ctx.close()


def test_replica_options_and_edits_apply_to_every_device(R, scenes):
    """rt_ctx_set_option and rt_update_lights / rt_update_materials reach every replica."""
    scene, prm, _ = scenes("C5", None)
    W, H = 64, 36
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    ctx = R.Context(scene, devices=[0, 0])
    try:
        ctx.set_option(R.OPT_KERNEL, R.KERNEL_WHOLE_TRAVERSAL)
        a, _ = ctx.render(cam, prm, W, H)
        ctx.set_option(R.OPT_KERNEL, R.KERNEL_AUTO)
        b, _ = ctx.render(cam, prm, W, H)
        assert a.tobytes() == b.tobytes()
        mats = scene.arrays()[3]
        edited = [R.material((0.1, 0.9, 0.2), m.ks, m.shininess, m.transparency) for m in mats]
        ctx.update_materials(edited, [R.material((0.5, 0.5, 0.5))])
        one = R.Context(scene)
        try:
            one.update_materials(edited, [R.material((0.5, 0.5, 0.5))])
            c1, _ = one.render(cam, prm, W, H)
        finally:
            one.close()
        c2, _ = ctx.render(cam, prm, W, H)
        assert c2.tobytes() == c1.tobytes()
        assert c2.tobytes() != b.tobytes()
    finally:
        ctx.close()


def test_create_rejects_bad_device_lists(R, scenes):
    scene, _, _ = scenes("C5", None)
    with pytest.raises(R.RtError, match="out of range"):
        R.Context(scene, devices=[0, 99])
    with pytest.raises(R.RtError, match="empty device list"):
        R.Context(scene, devices=[])


@pytest.mark.parametrize("mode", ["ipc", "ipc_fail_rank0", "none"])
def test_bench_ipc_exchange_two_processes(R, tmp_path, mode):
    """bench.py's N > 1 path, two ranks (gloo control plane, both on GPU 0).  ipc: rank 1's kernels store
    into rank 0's images; the result equals one process rendering the views.  ipc_fail_rank0: rank 0's
    IPC export fails (test hook) -- every rank still meets in the same collectives and the run falls back
    to the gather scheme with the same images.  none: the no-exchange control leg runs (each rank's bands
    into its own images)."""
    W, H, F = 160, 90, 3
    out = str(tmp_path / "imgs.npy")
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", PYTHONUNBUFFERED="1")
    if mode == "ipc_fail_rank0":
        env["BENCH_IPC_FAIL_RANK0"] = "1"
    port = {"ipc": 29511, "ipc_fail_rank0": 29512, "none": 29513}[mode]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1",
           "--warmup", "0", "--views", str(F), "--config", "C3", "--dragon-uv", "200x80", "--resolution",
           f"{W}x{H}", "--no-cpu-baseline", "--dump-images", out,
           "--exchange", "none" if mode == "none" else "ipc"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    if mode == "none":
        assert "NO exchange" in line, line
        return
    assert ("IPC-mapped" if mode == "ipc" else "all-gather") in line, line
    got = np.load(out)
    scene, prm, _, _, _ = R.build_config("C3", dragon_uv=(200, 80))
    ctx = R.Context(scene)
    try:
        ref, _ = ctx.render_views(R.turntable_cameras(F, R.aspect_of(W, H)), prm, W, H)
    finally:
        ctx.close()
    assert got.tobytes() == ref.tobytes()
