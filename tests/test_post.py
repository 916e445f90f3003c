"""Screen post-processing (src/screen.cpp): the CPU oracle (oracle/ref_post.cpp) against a
pure-Python loop restatement on tiny images, the BMP writer against the reference's own
render.bmp, and the HIP kernels (-m gpu) against the oracle.

Tolerances: bright-pass, box / Gaussian blur, clamp and Reinhard tone maps and the 8-bit
quantisation use the reference's exact op order and must be bit-identical; the exposure tone map
and gamma call expf / powf, where the device library may differ from glibc by <= 2 ulp, so they
are held to 1e-6 relative (well inside the 1e-5 absolute bar of BASELINE.json)."""
import gzip
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
F = np.float32


def hdr_image(W, H, seed):
    """Random HDR frame: mostly dim pixels, a few bright ones (so the bright-pass keeps some)."""
    rng = np.random.default_rng(seed)
    img = rng.uniform(0.0, 0.9, (H, W, 3)).astype(F)
    hot = rng.random((H, W)) < 0.15
    img[hot] = rng.uniform(0.8, 4.0, (int(hot.sum()), 3)).astype(F)
    return img.reshape(-1)


def py_bloom(img, W, H, opt, kernel, reps, fs, sigma, exposure):
    """applyBloomEffect in plain Python loops over float32 scalars (small images only)."""
    px = [tuple(F(v) for v in img[3 * k:3 * k + 3]) for k in range(W * H)]
    if opt == 0:
        return px
    wr, wg, wb = F(0.2126), F(0.7152), F(0.0722)
    light = [p if (p[0] * wr + p[1] * wg) + p[2] * wb >= F(1) else (F(0), F(0), F(0)) for p in px]
    reps = max(1, reps)
    sigma = max(F(0.001), F(sigma))

    def gw(x, y):
        a = 1.0 / (float(F(F(sigma * sigma) * F(2))) * 3.1415926535893238)
        e = F(math.exp(float(-(F(x * x) + F(y * y)) / F(F(F(2) * sigma) * sigma))))
        return F(a * float(e))

    def blur(src):
        out = []
        for y in range(H):
            for x in range(W):
                s = [F(0), F(0), F(0)]
                for i in range(-fs, fs + 1):
                    for j in range(-fs, fs + 1):
                        xx, yy = x + i, y + j
                        p = src[yy * W + xx] if 0 <= xx < W and 0 <= yy < H else (F(0), F(0), F(0))
                        w = gw(F(i), F(j)) if kernel == 1 else None
                        for c in range(3):
                            s[c] = F(s[c] + (F(w * p[c]) if kernel == 1 else p[c]))
                if kernel != 1:
                    n = F((2 * fs + 1) * (2 * fs + 1))
                    s = [F(v / n) for v in s]
                out.append(tuple(s))
        return out

    if opt == 4:
        return light
    if opt == 5:
        return blur(light)
    for _ in range(reps):
        light = blur(light)
    res = []
    for p, q in zip(px, light):
        v = [F(a + b) for a, b in zip(p, q)]
        if opt == 1:
            v = [min(max(a, F(0)), F(1)) for a in v]
        elif opt == 2:
            v = [F(a / F(a + F(1))) for a in v]
        res.append(tuple(v))
    return res


CASES = [  # (filtering option, kernel, repetitions, filter size, sigma)
    (1, 0, 1, 1, 2.0), (1, 1, 1, 2, 1.5), (2, 0, 2, 1, 2.0), (4, 0, 1, 1, 2.0), (5, 1, 1, 1, 0.7),
    (5, 0, 1, 0, 2.0), (1, 0, 1, -1, 2.0), (2, 1, 0, 1, 0.0),
]


@pytest.mark.parametrize("case", CASES)
def test_oracle_bloom_matches_python_loops(R, O, case):
    opt, kernel, reps, fs, sigma = case
    W, H = 7, 5
    img = hdr_image(W, H, 11)
    prm = R.post_params(filtering_option=opt, kernel=kernel, repetitions=reps, filter_size=fs, sigma=sigma)
    got, rgba = O.bitmap(img, W, H, prm)
    ref = np.array(py_bloom(img, W, H, opt, kernel, reps, fs, sigma, 0.5), F).reshape(-1)
    assert got.tobytes() == ref.tobytes()
    q = np.clip(ref.reshape(-1, 3), 0, 1) * F(255)
    assert np.array_equal(rgba.reshape(-1, 4)[:, :3], q.astype(np.uint8))
    assert (rgba.reshape(-1, 4)[:, 3] == 255).all()


def test_oracle_postprocess_gamma_only(R, O):
    W, H = 9, 4
    img = hdr_image(W, H, 3)
    prm = R.post_params(gamma_correction=True, gamma=2.2, filtering_option=1, bloom_live=False)
    got = O.postprocess(img, W, H, prm)
    ref = np.power(img, F(1) / F(2.2), dtype=F)  # bloom is not live: gamma only
    assert np.max(np.abs(got - ref) / np.maximum(ref, 1e-30)) <= 1e-6


def _read_bmp(raw):
    import struct

    off = struct.unpack_from("<I", raw, 10)[0]
    W, H = struct.unpack_from("<ii", raw, 18)
    bpp = struct.unpack_from("<H", raw, 28)[0]
    assert bpp == 24 and H > 0
    stride = (3 * W + 3) & ~3
    rgba = np.full((H, W, 4), 255, np.uint8)
    for r in range(H):  # bottom-up rows, BGR
        row = np.frombuffer(raw, np.uint8, 3 * W, off + (H - 1 - r) * stride).reshape(W, 3)
        rgba[r, :, :3] = row[:, ::-1]
    return W, H, rgba


def test_bmp_writer_reproduces_reference_render_bmp(R):
    """The reference's render.bmp (stbi_write_bmp output) decoded and re-encoded is byte-identical."""
    raw = gzip.open(os.path.join(GOLDEN, "render.bmp.gz")).read()
    W, H, rgba = _read_bmp(raw)
    assert R.encode_bmp(rgba.reshape(-1), W, H) == raw


def test_bmp_writer_row_padding(R, tmp_path):
    W, H = 5, 3  # 15 bytes per row -> 1 pad byte
    rgba = np.arange(W * H * 4, dtype=np.uint8)
    data = R.encode_bmp(rgba, W, H)
    assert len(data) == 54 + 16 * H
    w2, h2, back = _read_bmp(data)
    assert (w2, h2) == (W, H)
    assert np.array_equal(back[:, :, :3], rgba.reshape(H, W, 4)[:, :, :3])
    p = tmp_path / "x.bmp"
    R.check(R.lib().rt_write_bmp(str(p).encode(), W, H, rgba.ctypes.data_as(
        __import__("ctypes").POINTER(__import__("ctypes").c_uint8))), "rt_write_bmp")
    assert p.read_bytes() == data


GPU_CASES = CASES + [
    (3, 0, 1, 2, 2.0),  # exposure tone map (expf)
    (1, 0, 1, 20, 2.0),  # radius > 16: global-memory path
    (1, 1, 2, 17, 3.0),
    (0, 0, 1, 5, 2.0),
]


@pytest.mark.gpu
@pytest.mark.parametrize("case", GPU_CASES)
def test_gpu_bitmap_matches_oracle(R, O, case):
    opt, kernel, reps, fs, sigma = case
    W, H = 67, 45
    img = hdr_image(W, H, 5)
    prm = R.post_params(filtering_option=opt, kernel=kernel, repetitions=reps, filter_size=fs, sigma=sigma)
    got, rgba = R.bitmap(img, W, H, prm)
    ref, rref = O.bitmap(img, W, H, prm)
    if opt == 3:
        assert np.max(np.abs(got - ref)) <= 1e-6
        assert np.max(np.abs(rgba.astype(int) - rref.astype(int))) <= 1
    else:
        assert got.tobytes() == ref.tobytes()
        assert np.array_equal(rgba, rref)


@pytest.mark.gpu
@pytest.mark.parametrize("live,gamma", [(True, True), (False, True), (True, False)])
def test_gpu_postprocess_matches_oracle(R, O, live, gamma):
    W, H = 50, 37
    img = hdr_image(W, H, 9)
    prm = R.post_params(filtering_option=2, kernel=1, filter_size=3, sigma=1.2, bloom_live=live,
                        gamma_correction=gamma, gamma=1.8)
    got = R.postprocess(img, W, H, prm)
    ref = O.postprocess(img, W, H, prm)
    assert np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)) <= 1e-6


@pytest.mark.gpu
def test_gpu_bloom_full_hd_properties(R):
    """1920x1080: box blur of a constant bright image is the constant away from the border, and
    the quantised output of BLOOM (clamp) is 255 there."""
    W, H = 1920, 1080
    img = np.full(W * H * 3, 2.0, F)
    prm = R.post_params(filtering_option=5, kernel=0, filter_size=5)
    got, _ = R.bitmap(img, W, H, prm)
    v = got.reshape(H, W, 3)
    assert (v[5:-5, 5:-5] == F(2.0)).all()
    assert (v[0, 0] < F(2.0)).all()
    prm = R.post_params(filtering_option=1, kernel=0, filter_size=5)
    _, rgba = R.bitmap(img, W, H, prm)
    assert (rgba == 255).all()
