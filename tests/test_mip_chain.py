"""Mip levels past the chain (src/image.cpp:256-337, 478-486, 495-529).

getBestLevelMipmap clamps the ceil level to the chain but not the floor level, so a level of
detail at or past the number of mip levels picks a level getWidthHeightForLevel rejects: the
nearest-level filters then return white and trilinear returns black.  Both the oracle and the
device sampler follow that rule (neither indexes past the chain).  Known answers on a 4x4 texture
(levels 4, 2, 1) pin the oracle; the device sampler (rt_texture_sample) and a grazing-angle
textured render through rt_shade are compared with it."""
import os

import numpy as np
import pytest

WHITE, BLACK = (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)


def _png(path, w, h, value=None, seed=5):
    Image = pytest.importorskip("PIL.Image")
    if value is None:
        a = np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    else:
        a = np.full((h, w, 3), value, np.uint8)
    Image.fromarray(a, "RGB").save(path)


def _quad_scene(R, d, png, uv_scale=2.0):
    """A 2x2 quad in the y = 0 plane, uv running 0..uv_scale, kd texture `png`, a light above."""
    with open(os.path.join(d, "quad.obj"), "w") as f:
        f.write("mtllib quad.mtl\nv -1 0 -1\nv 1 0 -1\nv 1 0 1\nv -1 0 1\n")
        f.write(f"vt 0 0\nvt {uv_scale} 0\nvt {uv_scale} {uv_scale}\nvt 0 {uv_scale}\nvn 0 1 0\n")
        f.write("usemtl tex\nf 1/1/1 2/2/1 3/3/1 4/4/1\n")
    with open(os.path.join(d, "quad.mtl"), "w") as f:
        f.write(f"newmtl tex\nKd 1 1 1\nKs 0 0 0\nmap_Kd {png}\n")
    s = R.Scene()
    s.load_obj(os.path.join(d, "quad.obj"))
    s.add_point_light((0.0, 2.0, 0.0), (1.0, 1.0, 1.0))
    return s


def _prm(R, filt, oob=2):
    return R.params(max_reflection_level=0, glossy_ray_count=1, use_textures=True, texture_filtering=filt,
                    out_of_bounds_x=oob, out_of_bounds_y=oob, border_color=(0.2, 0.3, 0.4))


LODS = [0.0, 0.4, 0.6, 1.0, 1.49, 1.51, 2.0, 2.2, 2.5, 2.6, 2.99, 3.0, 3.2, 3.49, 3.5, 3.7, 4.0, 5.4, 5.6, 40.3,
        1e30, float(np.float32(3e38)), float("inf")]


def test_oracle_level_past_chain_known_answers(R, O, tmp_path):
    _png(str(tmp_path / "t4.png"), 4, 4)
    s = _quad_scene(R, str(tmp_path), "t4.png")
    o = O.Oracle(s)
    uv = np.array([[0.3, 0.7, lod] for lod in LODS], np.float32)
    near = o.texture_sample(0, uv, _prm(R, R.TEX_MIP_NEAREST))
    bil = o.texture_sample(0, uv, _prm(R, R.TEX_MIP_NEAREST_BILINEAR))
    tri = o.texture_sample(0, uv, _prm(R, R.TEX_TRILINEAR))
    for i, lod in enumerate(LODS):
        with np.errstate(invalid="ignore"):
            lower = (lod - np.floor(lod)) < (np.ceil(lod) - lod)  # mode 0 picks floor(lod); inf: NaN < NaN
        past_nearest = lower and np.floor(lod) >= 3  # 3 levels: 4x4, 2x2, 1x1
        past_tri = np.floor(lod) >= 3
        assert (tuple(near[i]) == WHITE) == past_nearest, lod  # random texels: never pure white
        assert (tuple(bil[i]) == WHITE) == past_nearest, lod
        assert (tuple(tri[i]) == BLACK) == past_tri, lod
    # a level past the chain is reached only through the floor level: lod 5.6 rounds up, clamps to 1x1
    i56 = LODS.index(5.6)
    assert tuple(near[i56]) != WHITE
    # a non-mipmappable texture: white for the nearest-level modes, black for trilinear (:256-258, :306-307)
    _png(str(tmp_path / "t35.png"), 3, 5)
    s2 = _quad_scene(R, str(tmp_path), "t35.png")
    o2 = O.Oracle(s2)
    assert (o2.texture_sample(0, uv, _prm(R, R.TEX_MIP_NEAREST)) == 1.0).all()
    assert (o2.texture_sample(0, uv, _prm(R, R.TEX_TRILINEAR)) == 0.0).all()


@pytest.mark.gpu
@pytest.mark.parametrize("size", [4, 8, 1])
def test_gpu_sampler_matches_oracle_across_the_chain(R, O, tmp_path, size):
    _png(str(tmp_path / "t.png"), size, size)
    s = _quad_scene(R, str(tmp_path), "t.png")
    ctx = R.Context(s)
    o = O.Oracle(s)
    rng = np.random.default_rng(11)
    lods = np.concatenate([np.array(LODS, np.float32), rng.uniform(0, 9, 400).astype(np.float32),
                           np.arange(0, 9, 0.25, dtype=np.float32)])
    uv = rng.uniform(-1.5, 2.5, (len(lods), 2)).astype(np.float32)
    q = np.concatenate([uv, lods[:, None]], axis=1)
    for filt in range(5):
        for oob in range(3):
            p = _prm(R, filt, oob)
            got = ctx.texture_sample(0, q, p)
            ref = o.texture_sample(0, q, p)
            assert got.tobytes() == ref.tobytes(), (filt, oob)
    ctx.close()


@pytest.mark.gpu
def test_gpu_grazing_render_past_the_chain(R, O, tmp_path):
    """getFinalColor on grazing rays over a black 4x4 texture: where the level of detail passes the
    chain the nearest-level filters shade with white kd, trilinear with black."""
    _png(str(tmp_path / "black.png"), 4, 4, value=0)
    s = _quad_scene(R, str(tmp_path), "black.png")
    ctx = R.Context(s)
    o = O.Oracle(s)
    xs, zs = np.meshgrid(np.linspace(-0.95, 0.95, 24), np.linspace(-0.95, 0.95, 24))
    targets = np.stack([xs.ravel(), np.zeros(xs.size), zs.ravel()], axis=1).astype(np.float32)
    rays = []
    for h, z0 in ((0.05, -3.0), (0.3, -2.0), (1.5, -0.5), (4.0, 0.0)):
        org = np.array([0.0, h, z0], np.float32)
        d = targets - org
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
        for t, dd in zip(targets, d):
            rays.append(((org[0], org[1], org[2]), tuple(dd), float(np.finfo(np.float32).max)))
    rays = np.array(rays, dtype=R.RAY_DTYPE)
    lit = {}
    for filt in (R.TEX_MIP_NEAREST, R.TEX_MIP_NEAREST_BILINEAR, R.TEX_TRILINEAR):
        p = _prm(R, filt)
        rgb, cnt = ctx.shade(rays, p)
        ref, rcnt = o.shade(rays, p)
        assert np.array_equal(cnt, rcnt), filt
        assert float(np.max(np.abs(rgb - ref))) <= 1e-5, filt
        lit[filt] = int((ref.max(axis=1) > 0).sum())
    # some rays land past the chain (white kd) and some do not (black texels)
    assert 0 < lit[R.TEX_MIP_NEAREST] < len(rays)
    assert lit[R.TEX_TRILINEAR] == 0
    ctx.close()
