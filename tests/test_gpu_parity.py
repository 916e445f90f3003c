"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the golden vectors.

Tolerance: every pixel within 1e-5 absolute of the oracle (BASELINE.json north_star); geometry
(t, hit points, normals, primitive ids, ray counts) must be bit-identical.  Full-size configs are
checked on sampled pixels plus size-independent properties (determinism, band-split invariance)."""
import os

import numpy as np
import pytest

import variants as V
from golden_cases import IMAGES, NATIVE_800, PRESET_IMAGES, apply

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.fixture(scope="module")
def ctxs(R):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    cache = {}

    def get(cfg, uv=None):
        key = (cfg, uv)
        if key not in cache:
            scene, prm, W, H, _ = R.build_config(cfg, dragon_uv=uv)
            cache[key] = (scene, R.Context(scene), prm, W, H)
        return cache[key]

    yield get
    for v in cache.values():
        v[1].close()


def golden(golden_dir):
    z = np.load(f"{golden_dir}/images.npz")
    out = {}
    for k in z.files:
        name, field = k.split("__")
        out.setdefault(name, {})[field] = z[k]
    return out


@pytest.mark.parametrize("case", IMAGES, ids=[c[0] for c in IMAGES])
def test_golden_images(R, ctxs, golden_dir, case):
    name, cfg, W, H, uv, over = case
    g = golden(golden_dir)[name]
    scene, ctx, prm, _, _ = ctxs(cfg, uv)
    prm = apply(R.rt_params.from_buffer_copy(prm), over)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    img, st = ctx.render(cam, prm, W, H)
    assert st.rays == int(g["rays"])
    assert float(np.max(np.abs(img - g["img"]))) <= TOL


@pytest.mark.parametrize("name,cfg", NATIVE_800, ids=[n for n, _ in NATIVE_800])
def test_native_800_frames(R, ctxs, golden_dir, name, cfg):
    """C1, C2 and C5 at renderRayTracing's native 800x800 (src/main.cpp:33) against the oracle's whole
    frames (tests/golden/native800.npz): every pixel within TOL, the same ray count."""
    z = np.load(f"{golden_dir}/native800.npz")
    _, ctx, prm, _, _ = ctxs(cfg)
    cam = R.camera_from_trackball(aspect=1.0)
    img, st = ctx.render(cam, prm, 800, 800)
    assert st.rays == int(z[f"{name}__rays"])
    assert float(np.max(np.abs(img - z[f"{name}__img"]))) <= TOL


@pytest.mark.parametrize("case", PRESET_IMAGES, ids=[c[0] for c in PRESET_IMAGES])
def test_golden_presets(R, golden_dir, case):
    name, preset, W, H, over = case
    g = golden(golden_dir)[name]
    scene = R.Scene().preset(R.PRESETS[preset], R.data_dir())
    ctx = R.Context(scene)
    prm = apply(R.params(), over)
    img, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), prm, W, H)
    ctx.close()
    assert st.rays == int(g["rays"])
    assert float(np.max(np.abs(img - g["img"]))) <= TOL


@pytest.mark.parametrize("cfg", ["C1", "C2", "C5"])
@pytest.mark.parametrize("use_bvh", [0, 1])
def test_intersect_kats_bit_exact(R, ctxs, golden_dir, cfg, use_bvh):
    z = np.load(f"{golden_dir}/kats.npz")
    _, ctx, _, _, _ = ctxs(cfg)
    hits = ctx.intersect(z[f"{cfg}__rays"], use_bvh)
    ref = z[f"{cfg}_bvh{use_bvh}__hits"]
    assert np.array_equal(hits["hit"], ref["hit"])
    assert hits["t"].tobytes() == ref["t"].tobytes()
    h = ref["hit"] == 1
    for f in ("normal", "hit_point", "material_index", "prim_id", "is_triangle"):
        assert hits[f][h].tobytes() == ref[f][h].tobytes(), f


@pytest.mark.parametrize("cfg", ["C2", "C5"])
def test_shade_matches_oracle(R, O, ctxs, golden_dir, cfg):
    """getFinalColor(level 0) on arbitrary rays (KAT rays: unit and non-unit directions)."""
    z = np.load(f"{golden_dir}/kats.npz")
    scene, ctx, prm, _, _ = ctxs(cfg)
    rays = z[f"{cfg}__rays"][:600]
    rgb, cnt = ctx.shade(rays, prm)
    ref, rcnt = O.Oracle(scene).shade(rays, prm)
    assert np.array_equal(cnt, rcnt)
    assert float(np.max(np.abs(rgb - ref))) <= TOL


def test_full_frame_c1_c2(R, O, ctxs):
    for cfg in ("C1", "C2"):
        scene, ctx, prm, W, H = ctxs(cfg)
        img, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), prm, W, H)
        ref, rays = O.Oracle(scene).render(prm, W, H)
        assert st.rays == rays, cfg
        assert float(np.max(np.abs(img - ref))) <= TOL, cfg


def _oracle_threads():
    """Host threads for the oracle: the box's CPU share (OMP_NUM_THREADS), not os.cpu_count()."""
    n = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return max(1, min(os.cpu_count() or 1, n if n > 0 else 16))


@pytest.mark.parametrize("cfg", ["C3", "C4", "C5"])
def test_full_size_sampled_pixels(R, O, ctxs, cfg):
    """Full BASELINE resolution on the GPU; BASELINE.md's CPU sample (4 096 pixels, the first 4 096
    of a seed-12345 permutation of the frame) re-rendered by the oracle, plus 64 pixels on
    geometry, every one within 1e-5."""
    scene, ctx, prm, W, H = ctxs(cfg)
    img, st = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), prm, W, H)
    assert np.isfinite(img).all()
    view = img.reshape(H, W, 3)[::-1]  # [y][x] in reference y order
    sel = np.random.default_rng(12345).permutation(W * H)[:4096]
    lit = np.argwhere(view.max(axis=2) > 0)
    pick = lit[np.random.default_rng(7).choice(len(lit), size=min(64, len(lit)), replace=False)]
    xy = np.concatenate([np.stack([sel % W, sel // W], axis=1), pick[:, ::-1]]).astype(np.int32)
    O.set_threads(_oracle_threads())
    ref, _, ub = O.Oracle(scene).render_pixels(prm, W, H, xy, with_ub=True)
    got = view[xy[:, 1], xy[:, 0]]
    assert float(np.max(np.abs(got - ref))) <= TOL
    if cfg in ("C3", "C4"):
        # the 800k-triangle proxy's triangles fall below barycentricCoordinates' 1e-4 area check:
        # the frame's shaded hits land in the reference's undefined regime (counted on both sides)
        R.set_counting(True)
        try:
            _, cst = ctx.render(R.camera_from_trackball(aspect=R.aspect_of(W, H)), prm, W, H)
        finally:
            R.set_counting(False)
        assert 0 < cst.ub_hits <= cst.hits
        assert int(ub.sum()) > 0


@pytest.mark.parametrize("cfg,uv,W,H", [("C2", None, 64, 48), ("C3", (200, 80), 96, 54), ("C4", (200, 80), 64, 36),
                                        ("C5", None, 64, 36)])
def test_ub_regime_count_matches_oracle(R, O, ctxs, cfg, uv, W, H):
    """The counting build's ub_hits (shaded triangle hits where the reference's
    barycentricCoordinates returns false and it interpolates uninitialised coordinates,
    src/ray_tracing.cpp:147-157, 281-295) equals the oracle's count over the whole frame."""
    scene, ctx, prm, _, _ = ctxs(cfg, uv)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    R.set_counting(True)
    try:
        img, st = ctx.render(cam, prm, W, H)
    finally:
        R.set_counting(False)
    xs, ys = np.meshgrid(np.arange(W), np.arange(H))
    xy = np.stack([xs.ravel(), ys.ravel()], axis=1).astype(np.int32)
    O.set_threads(_oracle_threads())
    _, rays, ub = O.Oracle(scene).render_pixels(prm, W, H, xy, with_ub=True)
    assert st.rays == int(rays.sum())
    assert st.ub_hits == int(ub.sum())
    assert st.ub_hits <= st.hits


@pytest.mark.parametrize("cfg,uv", [("C3", (200, 80)), ("C4", (200, 80)), ("C5", None)])
def test_band_split_bit_identical(R, ctxs, cfg, uv):
    """The multi-GPU layout (interleaved 8-row bands per rank + un-permute) reproduces the
    single-GPU frame bit for bit, and a re-render is deterministic."""
    import ctypes

    import torch

    scene, ctx, prm, _, _ = ctxs(cfg, uv)
    W, H = 200, 123
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    full, st = ctx.render(cam, prm, W, H)
    again, _ = ctx.render(cam, prm, W, H)
    assert full.tobytes() == again.tobytes()
    for count in (2, 3, 8):
        n = R.local_band_elems(W, H, 8, count)
        gathered = torch.zeros(count * n, dtype=torch.float32, device="cuda")
        rays = 0
        for rank in range(count):
            part = gathered[rank * n:(rank + 1) * n]
            s = ctx.render_device(cam, prm, W, H, 8, rank, count, part.data_ptr(), None)
            rays += s.rays
        torch.cuda.synchronize()
        img = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        R.check(R.lib().rt_unpermute_bands_device(W, H, 8, count, ctypes.c_void_p(gathered.data_ptr()),
                                                  ctypes.c_void_p(img.data_ptr()), None))
        torch.cuda.synchronize()
        assert img.cpu().numpy().tobytes() == full.tobytes()
        host = R.unpermute_host(gathered.cpu().numpy(), W, H, 8, count)
        assert host.tobytes() == full.tobytes()
        assert rays == st.rays


@pytest.mark.parametrize("cfg,uv", [("C3", (200, 80)), ("C4", (200, 80)), ("C2", None)])
def test_band_split_view_batch_bit_identical(R, ctxs, cfg, uv):
    """bench.py's N>1 step on one GPU: each rank's bands of every view in one launch, the buffers
    back to back as all_gather_into_tensor leaves them, one rt_unpermute_views_device launch --
    every view bit-identical to rt_render_views, ray counts add up."""
    import ctypes

    import torch

    scene, ctx, prm, _, _ = ctxs(cfg, uv)
    W, H, F = 120, 67, 3
    cams = R.turntable_cameras(F, R.aspect_of(W, H))
    ref, rst = ctx.render_views(cams, prm, W, H)
    for count in (2, 3):
        n = F * R.local_band_elems(W, H, 8, count)
        gathered = torch.full((count * n,), -1.0, dtype=torch.float32, device="cuda")
        rays = 0
        for rank in range(count):
            part = gathered[rank * n:(rank + 1) * n]
            rays += ctx.render_views_device(cams, prm, W, H, 8, rank, count, part.data_ptr(), None).rays
        imgs = torch.zeros(F * W * H * 3, dtype=torch.float32, device="cuda")
        R.check(R.lib().rt_unpermute_views_device(W, H, 8, count, F, ctypes.c_void_p(gathered.data_ptr()),
                                                  ctypes.c_void_p(imgs.data_ptr()), None))
        torch.cuda.synchronize()
        got = imgs.cpu().numpy().reshape(F, -1)
        assert got.tobytes() == ref.tobytes(), count
        assert R.unpermute_views_host(gathered.cpu().numpy(), W, H, 8, count, F).tobytes() == ref.tobytes()
        assert rays == rst.rays


def test_device_math_is_ieee(R, ctxs):
    _, ctx, _, _, _ = ctxs("C1")
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(1e-6, 10, 20000), rng.uniform(-1, 1, 20000)]).astype(np.float32)
    x[x == 0] = 1.0
    y = rng.uniform(-4, 250, len(x)).astype(np.float32)
    out = ctx.selftest_math(x, y)
    with np.errstate(all="ignore"):
        pos = x > 0
        assert out[pos, 0].tobytes() == np.sqrt(x[pos]).tobytes()  # correctly rounded sqrt
        assert out[:, 1].tobytes() == (np.float32(1) / x).tobytes()  # correctly rounded division
        assert out[:, 2].tobytes() == (x / y).tobytes()
        ref = np.power(x[pos].astype(np.float64), y[pos].astype(np.float64)).astype(np.float32)
        got = out[pos, 3]
        fin = np.isfinite(ref) & (ref != 0)
        ulp = np.abs(got[fin].view(np.int32).astype(np.int64) - ref[fin].view(np.int32).astype(np.int64))
        assert ulp.max() <= 2  # powf feeds colours only (calcColor specular)


def test_invalid_params_fail_loudly(R, ctxs):
    _, ctx, prm, _, _ = ctxs("C1")
    bad = R.params(max_reflection_level=99, glossy_ray_count=1)
    with pytest.raises(R.RtError, match="max_reflection_level"):
        ctx.render(R.camera_from_trackball(), bad, 8, 8)


@pytest.mark.parametrize("case", ["c2_64x48", "c3s_96x54", "c4s_64x36", "c5_96x54", "c5_depth3_bvh_64x36"])
def test_kernel_variants_bit_identical(R, ctxs, golden_dir, case):
    """Every render path (whole-traversal / dynamic-fetch kernels, each compiled variant, drain lane
    groups and refill thresholds) gives the same bits and ray count, and matches the golden image."""
    name, cfg, W, H, uv, over = next(c for c in IMAGES if c[0] == case)
    g = golden(golden_dir)[name]
    _, ctx, prm, _, _ = ctxs(cfg, uv)
    prm = apply(R.rt_params.from_buffer_copy(prm), over)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    base = None
    for v in V.all_variants(R):
        with V.options(R, ctx, v):
            img, st = ctx.render(cam, prm, W, H)
        assert st.rays == int(g["rays"]), v
        assert float(np.max(np.abs(img - g["img"]))) <= TOL, v
        if base is None:
            base = img
        assert img.tobytes() == base.tobytes(), v


@pytest.mark.parametrize("cfg,uv,kernel,aa", [("C2", None, "", 0), ("C2", None, "df", 0), ("C2", None, "df", 1),
                                              ("C3", (200, 80), "", 0), ("C3", (200, 80), "tail", 0),
                                              ("C3", (200, 80), "wf", 0), ("C2", None, "wf", 0),
                                              ("C3", (200, 80), "split", 0), ("C3", (200, 80), "split", 1),
                                              ("C4", (200, 80), "", 0), ("C5", None, "", 0)])
def test_view_batch_bit_identical(R, O, ctxs, cfg, uv, kernel, aa):
    """rt_render_views_device: every view of a batch is bit-identical to rt_render_device with that
    camera (whole frame and band ranks; the batch runs its own refill / lane-group defaults), ray
    counts add up, and a rotated view matches the oracle."""
    import torch

    scene, ctx, prm, _, _ = ctxs(cfg, uv)
    opts = {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH} if kernel == "df" else {}
    if kernel == "tail":  # the opaque kernel with the batch's last two views interleaved over 16 tiles
        opts = {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_INTERLEAVE_TAIL: 2}
    if kernel == "wf":  # the wavefront path (trace / shade kernels per recursion level)
        opts = {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_WAVEFRONT: 1}
    if kernel == "split":  # the opaque kernel with the shadow segments traced beside the mirror chain
        opts = {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_OPAQUE: 4}
    with V.options(R, ctx, opts):
        _view_batch_checks(R, O, scene, ctx, prm, cfg, aa)


def _view_batch_checks(R, O, scene, ctx, prm, cfg, aa):
    import torch

    if aa:
        prm = type(prm).from_buffer_copy(prm)
        prm.anti_aliasing = 1
    W, H = 100, 61  # ragged: a partial 8x8 tile column and a partial band
    cams = R.turntable_cameras(5, R.aspect_of(W, H))
    for rank, count in ((0, 1), (1, 3)):
        n = R.local_band_elems(W, H, 8, count)
        batch = torch.full((len(cams) * n,), -1.0, dtype=torch.float32, device="cuda")
        st = ctx.render_views_device(cams, prm, W, H, 8, rank, count, batch.data_ptr(), None)
        torch.cuda.synchronize()
        rays = 0
        for v, cam in enumerate(cams):
            one = torch.full((n,), -1.0, dtype=torch.float32, device="cuda")
            s = ctx.render_device(cam, prm, W, H, 8, rank, count, one.data_ptr(), None)
            torch.cuda.synchronize()
            rays += s.rays
            assert batch[v * n:(v + 1) * n].cpu().numpy().tobytes() == one.cpu().numpy().tobytes(), (v, rank)
        assert st.rays == rays
    host, sth = ctx.render_views(cams, prm, W, H)  # rt_render_views: host output, rt_render layout
    hrays = 0
    for v, cam in enumerate(cams):
        one, s = ctx.render(cam, prm, W, H)
        hrays += s.rays
        assert host[v].tobytes() == one.tobytes(), v
    assert sth.rays == hrays
    img, st1 = ctx.render(cams[2], prm, W, H)
    ref, rays = O.Oracle(scene).render(prm, W, H, euler=R.turntable_eulers(5)[2])
    assert st1.rays == rays
    assert float(np.max(np.abs(img - ref))) <= TOL


def test_sphere_light_fans_match_oracle(R, O, ctxs):
    """Spherical-light samples traced as wave-shared fans (dynamic-fetch kernel, opaque scene) give
    the per-lane loop's bits and ray counts, for frames and for rt_shade's explicit rays (whose
    per-ray counts include the fan samples other lanes traced), and match the oracle."""
    scene, ctx, prm, _, _ = ctxs("C4", (200, 80))
    W, H = 64, 36
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    out = {}
    for fan in (1, 0):
        with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_FAN: fan}):
            out[fan] = ctx.render(cam, prm, W, H)
    assert out[1][0].tobytes() == out[0][0].tobytes()
    assert out[1][1].rays == out[0][1].rays
    ref, rays = O.Oracle(scene).render(prm, W, H)
    assert out[1][1].rays == rays
    assert float(np.max(np.abs(out[1][0] - ref))) <= TOL
    # rt_shade: 256 rays from one eye point towards random points around the model, level 0
    rng = np.random.default_rng(5)
    rays_in = np.zeros(256, R.RAY_DTYPE)
    hits = rng.uniform(-0.4, 0.4, (len(rays_in), 3)).astype(np.float32)
    rays_in["origin"] = np.float32([0.0, 0.2, -3.0])
    dirs = hits - rays_in["origin"]
    rays_in["direction"] = dirs / np.linalg.norm(dirs, axis=1, keepdims=True)
    rays_in["t"] = np.float32(np.finfo(np.float32).max)
    got = {}
    for fan in (1, 0):
        with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_FAN: fan}):
            got[fan] = ctx.shade(rays_in, prm)
    assert got[1][0].tobytes() == got[0][0].tobytes()
    assert np.array_equal(got[1][1], got[0][1])
    rgb_ref, cnt_ref = O.Oracle(scene).shade(rays_in, prm)
    assert np.array_equal(got[1][1], cnt_ref)
    assert float(np.max(np.abs(got[1][0] - rgb_ref))) <= TOL


def test_plane_and_transparent_fans_match_oracle(R, O):
    """Plane-light grids and spherical lights in a scene with a transparent (glass) sphere, traced as
    wave-shared fans: each sample runs its own cansee segment loop and hands back its intensity, and
    the owner sums them in the loop's order -- the per-lane loop's bits and ray counts, and the oracle,
    for frames and rt_shade."""
    scene, prm, _, _, _ = R.build_config("C5")
    scene.add_spherical_light((0.05, 0.5, 0.1), 0.08, (0.5, 0.5, 0.5))
    prm.max_reflection_level = 3
    prm.sphere_light_ray_count = 37
    ctx = R.Context(scene)
    try:
        W, H = 48, 32
        cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
        out = {}
        for fan in (1, 0):
            with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_FAN: fan}):
                out[fan] = ctx.render(cam, prm, W, H)
        assert out[1][0].tobytes() == out[0][0].tobytes()
        assert out[1][1].rays == out[0][1].rays
        ref, rays = O.Oracle(scene).render(prm, W, H)
        assert out[1][1].rays == rays
        assert float(np.max(np.abs(out[1][0] - ref))) <= TOL
        # rt_shade through the glass sphere and the box
        rng = np.random.default_rng(11)
        rays_in = np.zeros(192, R.RAY_DTYPE)
        tgt = rng.uniform(-0.5, 0.5, (len(rays_in), 3)).astype(np.float32)
        rays_in["origin"] = np.float32([0.0, 0.0, 2.5])
        dirs = tgt - rays_in["origin"]
        rays_in["direction"] = dirs / np.linalg.norm(dirs, axis=1, keepdims=True)
        rays_in["t"] = np.float32(np.finfo(np.float32).max)
        got = {}
        for fan in (1, 0):
            with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_FAN: fan}):
                got[fan] = ctx.shade(rays_in, prm)
        assert got[1][0].tobytes() == got[0][0].tobytes()
        assert np.array_equal(got[1][1], got[0][1])
        rgb_ref, cnt_ref = O.Oracle(scene).shade(rays_in, prm)
        assert np.array_equal(got[1][1], cnt_ref)
        assert float(np.max(np.abs(got[1][0] - rgb_ref))) <= TOL
    finally:
        ctx.close()


def test_c4_full_size_batch_four_wave_tree(R, ctxs):
    """The batch that faulted the 4-wave recursion-tree build in rounds 4-5: C4 at 1920x1080, a 16-view turntable in
    one launch.  The shipped batch build (4 waves, every automatic variable defined: build.py HIP_FLAGS) renders the
    same bits and ray count as the 3-wave build (RT_OPT_TREE 5) and as single frames of the same cameras."""
    import torch

    scene, ctx, prm, W, H = ctxs("C4")
    F = 16
    cams = R.turntable_cameras(F, R.aspect_of(W, H))
    out = {}
    for tree in (-1, 5):
        buf = torch.full((F * W * H * 3,), -1.0, dtype=torch.float32, device="cuda")
        with V.options(R, ctx, {R.OPT_TREE: tree}):
            st = ctx.render_views_image_device(cams, prm, W, H, buf.data_ptr(), None)
        torch.cuda.synchronize()
        out[tree] = (buf, st.rays, st.kernel_name)
    assert "persistent_tree_kernel<false, 18>" in out[-1][2], out[-1][2]
    assert "persistent_tree_kernel<false, 10>" in out[5][2], out[5][2]
    assert out[-1][1] == out[5][1]
    assert torch.equal(out[-1][0], out[5][0])
    one, _ = ctx.render(cams[5], prm, W, H)
    assert out[-1][0].view(F, -1)[5].cpu().numpy().tobytes() == one.tobytes()


def test_bench_step_c3_64_views(R, O, ctxs):
    """The benchmarked step itself (bench.py defaults): C3 at 1920x1080, a 64-view turntable in ONE
    rt_render_views_device launch, rebuilt by rt_unpermute_views_device.  Views 0, 21 and 63 are
    bit-identical to single-frame renders with their cameras; the batch's ray count is the sum of the
    64 single-frame counts; 256 pixels of view 21 (half of them on geometry) match the oracle."""
    import torch

    scene, ctx, prm, W, H = ctxs("C3")
    F = 64
    eulers = R.turntable_eulers(F)
    cams = [R.camera_from_trackball(euler=e, aspect=R.aspect_of(W, H)) for e in eulers]
    n = R.local_band_elems(W, H, 8, 1)
    local = torch.full((F * n,), -1.0, dtype=torch.float32, device="cuda")
    images = torch.full((F * W * H * 3,), -1.0, dtype=torch.float32, device="cuda")
    import time
    t0 = time.time()
    st = ctx.render_views_device(cams, prm, W, H, 8, 0, 1, local.data_ptr(), None)
    print(f"bench step: batch {time.time() - t0:.2f} s, kernel {st.kernel_ms:.1f} ms", flush=True)
    R.check(R.lib().rt_unpermute_views_device(W, H, 8, 1, F, R.C.c_void_p(local.data_ptr()),
                                              R.C.c_void_p(images.data_ptr()), R.C.c_void_p(0)), "unpermute")
    torch.cuda.synchronize()
    imgs = images.view(F, H * W * 3)
    rays = 0
    for v, cam in enumerate(cams):
        one, s1 = ctx.render(cam, prm, W, H)
        rays += s1.rays
        if v in (0, 21, 63):
            got = imgs[v].cpu().numpy()
            bad = np.nonzero(got != one)[0]
            assert len(bad) == 0, (v, len(bad), bad[:8].tolist(), float(np.max(np.abs(got - one))), s1.kernel_name,
                                   st.kernel_name)
    assert st.rays == rays
    print(f"bench step: single frames done {time.time() - t0:.2f} s", flush=True)
    view = imgs[21].cpu().numpy().reshape(H, W, 3)[::-1]  # [y][x], reference y order
    lit = np.argwhere(view.max(axis=2) > 0)
    pick = lit[np.random.default_rng(21).choice(len(lit), size=128, replace=False)][:, ::-1]
    sel = np.random.default_rng(5).permutation(W * H)[:128]
    xy = np.concatenate([np.stack([sel % W, sel // W], axis=1), pick]).astype(np.int32)
    O.set_threads(_oracle_threads())
    ref, _ = O.Oracle(scene).render_pixels(prm, W, H, xy, euler=eulers[21])
    print(f"bench step: oracle done {time.time() - t0:.2f} s", flush=True)
    assert float(np.max(np.abs(view[xy[:, 1], xy[:, 0]] - ref))) <= TOL


@pytest.mark.parametrize("depth,multi", [(0, 0), (9, 0), (15, 0), (4, 4)])
def test_split_depths_and_samples(R, O, depth, multi):
    """SPLIT at the recursion depths its frame and LDS result bits span (a lone level-0 node; ten levels; level 15,
    the deepest rt_params accepts, RT_MAX_DEPTH - 1: the top LDS result bit and the 4-bit level field) and with
    getPixelRays' 4 samples per pixel (each sample folded and stored in sample order, store_sample): the SPLIT
    builds against the opaque kernel without SPLIT and the oracle (bits, ray count)."""
    scene, prm, _, _, _ = R.build_config("C3", dragon_uv=(200, 80))
    prm = type(prm).from_buffer_copy(prm)
    prm.max_reflection_level = depth
    if multi:
        prm.multiple_rays = 1
        prm.sample_size = multi
    W, H = 64, 36
    ctx = R.Context(scene)
    try:
        cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
        ref, rays = O.Oracle(scene).render(prm, W, H)
        base = None
        for opaque in (1, 4, 5):
            with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_OPAQUE: opaque}):
                img, st = ctx.render(cam, prm, W, H)
            assert st.rays == rays, opaque
            assert float(np.max(np.abs(img - ref))) <= TOL, opaque
            if base is None:
                base = img
            assert img.tobytes() == base.tobytes(), opaque
    finally:
        ctx.close()


@pytest.mark.gpu
def test_split_single_spot_light(R, O):
    """SPLIT (rt_megakernel.hip split_node) with its one light a spot light: split_light's cone test decides
    whether a node posts a segment (inside the cone) or keeps a zero colour (outside, src/shadow.cpp:235-237).  The
    dragon proxy lit by one narrow spot light only, every SPLIT build against the general kernels, the opaque
    kernel without SPLIT and the oracle (bits, ray count)."""
    scene, prm, _, _, _ = R.build_config("C3", dragon_uv=(200, 80))
    scene.clear_lights()
    scene.add_spot_light((1, 1, -1), (-1, -1, 1), 15, (0.9, 0.7, 0.5))
    W, H = 96, 54
    ctx = R.Context(scene)
    try:
        cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
        ref, rays = O.Oracle(scene).render(prm, W, H)
        base = None
        for opaque in (0, 1, 4, 5, 7):
            with V.options(R, ctx, {R.OPT_KERNEL: R.KERNEL_DYNAMIC_FETCH, R.OPT_OPAQUE: opaque}):
                img, st = ctx.render(cam, prm, W, H)
            assert st.rays == rays, opaque
            assert float(np.max(np.abs(img - ref))) <= TOL, opaque
            if base is None:
                base = img
            assert img.tobytes() == base.tobytes(), opaque
        assert float(np.abs(ref).max()) > 0.0  # the cone lights part of the object
    finally:
        ctx.close()


def test_opaque_kernel_spot_lights(R, O):
    """Spot lights through the opaque-scene kernel (lite_next_light's cone test and its point-then-spot
    light order, rt_megakernel.hip) against the general kernels and the oracle: the dragon proxy lit by one
    point light and two spot lights whose cones cut the object (src/shadow.cpp:228-247), so pixels inside
    and outside each cone occur.  Every build of the opaque kernel (4-wave, 3-wave, the re-visit group
    stack) renders the general kernels' bits and ray count."""
    scene, prm, _, _, _ = R.build_config("C3", dragon_uv=(200, 80))
    scene.clear_lights()
    scene.add_point_light((-1, 1, -1), (0.5, 0.5, 0.5))
    scene.add_spot_light((1, 1, -1), (-1, -1, 1), 20, (0.8, 0.6, 0.4))
    scene.add_spot_light((0, 1.5, 0.2), (0, -1, -0.1), 10, (0.3, 0.3, 0.9))
    W, H = 96, 54
    ctx = R.Context(scene)
    try:
        cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
        ref, rays = O.Oracle(scene).render(prm, W, H)
        df = R.KERNEL_DYNAMIC_FETCH
        base = None
        for opaque, refill in ((0, 0), (1, 0), (2, 0), (3, 0)):
            with V.options(R, ctx, {R.OPT_KERNEL: df, R.OPT_OPAQUE: opaque, R.OPT_REFILL: refill}):
                img, st = ctx.render(cam, prm, W, H)
            assert ("opaque" in st.kernel_name) == (opaque != 0), (opaque, st.kernel_name)
            assert st.rays == rays, opaque
            assert float(np.max(np.abs(img - ref))) <= TOL, opaque
            if base is None:
                base = img
            assert img.tobytes() == base.tobytes(), opaque
        # the spot lights light part of the object: without them the image changes, but not everywhere
        point_only, _, _, _, _ = R.build_config("C3", dragon_uv=(200, 80))
        point_only.clear_lights()
        point_only.add_point_light((-1, 1, -1), (0.5, 0.5, 0.5))
        diff = np.any(O.Oracle(point_only).render(prm, W, H)[0].reshape(-1, 3) != ref.reshape(-1, 3), axis=1)
        assert 0 < int(diff.sum()) < W * H
    finally:
        ctx.close()
