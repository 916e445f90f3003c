"""kd textures (useTextures, src/main.cpp:146-171): PNG ingest with stbi_load(..., STBI_rgb)
semantics (src/image.cpp:37-73), the mip chain (:408-452), getPixel's out-of-bounds rules and
five filters (:77-360), and the ray-differential level of detail (src/ray_differentials.cpp).

Pins: the PNG decoder against PIL (an independent decoder) on the reference's own texture
files and on synthetic files of every colour type; the GPU against the oracle restatement
(oracle/ref_cpu.cpp, struct Image / level_of_detail) on the reference's checker scene
(data/checker.obj, UVs outside [0,1]) with a mirror sphere above it, so camera and secondary
rays both sample.  Ray counts equal, pixels within 1e-5.  The mipmap levels of detail rest on
Ray's member initialisers as intended (right = (1,0,0), up = (0,-1,0)); the reference reads
them uninitialised (framework/include/ray.h:19-20), so for the three mipmap filters parity
against the reference binary itself is unpinned."""
import io
import os
import shutil

import numpy as np
import pytest

FIXTURE_PNGS = ["default.png", "bookshelf.png", "green_wool.png", "stone_bricks.png"]


def _pil():
    return pytest.importorskip("PIL.Image")


def _pil_channels(im):
    if im.mode == "P":
        return 4 if "transparency" in im.info else 3
    return {"L": 1, "1": 1, "LA": 2, "RGB": 3, "RGBA": 4, "I;16": 1, "I;16B": 1}[im.mode]


@pytest.mark.parametrize("name", FIXTURE_PNGS)
def test_png_decode_matches_pil_on_reference_textures(R, name):
    Image = _pil()
    path = os.path.join(R.data_dir(), name)
    data = open(path, "rb").read()
    rgb, ch = R.decode_png(data)
    im = Image.open(io.BytesIO(data))
    assert ch == _pil_channels(im)
    assert np.array_equal(rgb, np.asarray(im.convert("RGB")))


@pytest.mark.parametrize("mode", ["1", "L", "LA", "RGB", "RGBA", "P", "I;16"])
def test_png_decode_colour_types(R, mode):
    Image = _pil()
    rng = np.random.default_rng(7)
    H, W = 13, 17
    if mode == "I;16":
        a = rng.integers(0, 65536, (H, W), dtype=np.uint16)
        im = Image.fromarray(a)
        assert im.mode.startswith("I;16")
        want = np.repeat((a >> 8).astype(np.uint8)[..., None], 3, axis=2)  # stb keeps the high byte
    else:
        base = rng.integers(0, 256, (H, W, 4), dtype=np.uint8)
        im = Image.fromarray(base, "RGBA").convert(mode)
        want = np.asarray(im.convert("RGB"))
    buf = io.BytesIO()
    im.save(buf, "PNG")
    rgb, ch = R.decode_png(buf.getvalue())
    assert ch == _pil_channels(Image.open(io.BytesIO(buf.getvalue())))
    assert np.array_equal(rgb, want)


def _textured_scene(R, tmp, png, sphere=True):
    """data/checker.obj with its material's map_Kd pointing at `png`, a point light above and
    (optionally) a mirror sphere whose reflections land on the textured floor."""
    dd = R.data_dir()
    obj = open(os.path.join(dd, "checker.obj")).read().replace("mtllib checker3.mtl", "mtllib tex.mtl")
    mtl = open(os.path.join(dd, "checker3.mtl")).read().replace("map_Kd default.png", f"map_Kd {png}")
    with open(os.path.join(tmp, "checker.obj"), "w") as f:
        f.write(obj)
    with open(os.path.join(tmp, "tex.mtl"), "w") as f:
        f.write(mtl)
    if os.path.exists(os.path.join(dd, png)):
        shutil.copy(os.path.join(dd, png), os.path.join(tmp, png))
    s = R.Scene()
    s.load_obj(os.path.join(tmp, "checker.obj"))
    s.add_point_light((0.0, 2.0, 1.0), (1.0, 1.0, 1.0))
    if sphere:
        s.add_sphere((0.0, 0.45, -0.5), 0.4, R.material(kd=(0.1, 0.1, 0.1), ks=(0.8, 0.8, 0.8), shininess=0.0))
    return s


def _params(R, filt, oob_x, oob_y, depth=2):
    return R.params(max_reflection_level=depth, glossy_ray_count=1, use_textures=True, texture_filtering=filt,
                    out_of_bounds_x=oob_x, out_of_bounds_y=oob_y, border_color=(0.2, 0.3, 0.4))


def test_texture_ingest_errors(R, tmp_path):
    Image = _pil()
    Image.fromarray(np.zeros((4, 4), np.uint8), "L").save(tmp_path / "grey.png")
    with pytest.raises(R.RtError, match="3 or more color channels"):
        _textured_scene(R, str(tmp_path), "grey.png")
    with pytest.raises(R.RtError, match="does not exist"):
        _textured_scene(R, str(tmp_path), "missing.png")


def test_oracle_texture_rules_and_filters(R, O, tmp_path):
    """The oracle's getPixel behaves as the reference's rules say on the checker floor (UVs run
    to -1.4..2.4): Border shows the border colour, Clamp / Repeat do not, filters differ."""
    s = _textured_scene(R, str(tmp_path), "green_wool.png", sphere=False)
    W, H = 40, 24
    o = O.Oracle(s)
    plain, r0 = o.render(R.params(max_reflection_level=0, glossy_ray_count=1), W, H)
    imgs = {}
    for filt in range(5):
        for oob in range(3):
            img, r = o.render(_params(R, filt, oob, oob, depth=0), W, H)
            assert r == r0  # textures never change the ray tree
            imgs[(filt, oob)] = img
    assert float(np.abs(imgs[(0, 1)] - plain).max()) > 0.05
    assert float(np.abs(imgs[(0, 0)] - imgs[(0, 1)]).max()) > 0.05
    assert float(np.abs(imgs[(0, 1)] - imgs[(0, 2)]).max()) > 0.05
    assert float(np.abs(imgs[(0, 2)] - imgs[(1, 2)]).max()) > 0.01
    assert float(np.abs(imgs[(1, 2)] - imgs[(4, 2)]).max()) > 0.01


def _compare_gpu(R, O, s, cases, W=48, H=32, kernels=("whole", "df")):
    import variants as V

    ctx = R.Context(s)
    o = O.Oracle(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    kinds = {"whole": R.KERNEL_WHOLE_TRAVERSAL, "df": R.KERNEL_DYNAMIC_FETCH}
    for p in cases:
        ref, rays = o.render(p, W, H)
        for k in kernels:
            with V.options(R, ctx, {R.OPT_KERNEL: kinds[k]}):
                img, st = ctx.render(cam, p, W, H)
            tag = (k, p.texture_filtering, p.out_of_bounds_x, p.out_of_bounds_y)
            assert st.rays == rays, tag
            assert float(np.max(np.abs(img - ref))) <= 1e-5, tag
    ctx.close()


@pytest.mark.gpu
def test_gpu_textures_every_filter_and_rule(R, O, tmp_path):
    s = _textured_scene(R, str(tmp_path), "green_wool.png")
    cases = [_params(R, f, ox, oy) for f in range(5) for (ox, oy) in [(0, 0), (1, 1), (2, 2), (2, 1)]]
    _compare_gpu(R, O, s, cases)


@pytest.mark.gpu
@pytest.mark.parametrize("png", ["default.png", "bookshelf.png", "stone_bricks.png"])
def test_gpu_textures_reference_files(R, O, tmp_path, png):
    s = _textured_scene(R, str(tmp_path), png)
    cases = [_params(R, f, 2, 2) for f in (0, 1, 4)]
    _compare_gpu(R, O, s, cases, kernels=("whole", "df"))


@pytest.mark.gpu
def test_gpu_textures_off_is_untextured(R, O, tmp_path):
    s = _textured_scene(R, str(tmp_path), "green_wool.png")
    p = R.params(max_reflection_level=2, glossy_ray_count=1)
    _compare_gpu(R, O, s, [p], kernels=("df",))
