"""Glossy lobes (glossy_ray_count > 1, src/main.cpp:204-250).  The reference draws the lobe
directions with rand(); this build defines that stream as Philox-4x32-10 keyed by
rt_params.rng_seed with counter (draw, pixel, sample, 0), shared by the GPU and the oracle
(DESIGN.md section 3).  Parity therefore holds per seed: ray counts equal, pixels within 1e-5
(the only device/host difference is powf in the lobe weight, <= 2 ulp)."""
import ctypes as C

import numpy as np
import pytest

# Random123 known-answer vectors for philox4x32_10 (ctr, key, expected)
KATS = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def _u32(v):
    return (C.c_uint32 * len(v))(*v)


@pytest.mark.parametrize("ctr,key,want", KATS)
def test_philox_known_answers(R, O, ctr, key, want):
    out = _u32([0] * 4)
    R.check(R.lib().rt_philox4x32_10(_u32(ctr), _u32(key), out), "rt_philox4x32_10")
    assert tuple(out) == want
    out2 = _u32([0] * 4)
    O.lib().oracle_philox(_u32(ctr), _u32(key), out2)
    assert tuple(out2) == want


def _cornell(R, glossy, seed, depth=3):
    s, p, _, _, _ = R.build_config("C5")
    p.glossy_ray_count = glossy
    p.rng_seed = seed
    p.max_reflection_level = depth
    return s, p


def test_oracle_glossy_is_seeded(R, O):
    s, p = _cornell(R, 6, 0x5EED)
    W, H = 24, 14
    xy = np.array([[x, y] for y in range(4, 10) for x in range(6, 18)], np.int32)
    o = O.Oracle(s)
    a, ra = o.render_pixels(p, W, H, xy)
    b, rb = o.render_pixels(p, W, H, xy)
    assert a.tobytes() == b.tobytes() and np.array_equal(ra, rb)
    p.rng_seed = 0x1234
    c, rc = o.render_pixels(p, W, H, xy)
    assert not (a.tobytes() == c.tobytes() and np.array_equal(ra, rc))
    p.glossy_ray_count = 1
    d, rd = o.render_pixels(p, W, H, xy)
    assert int(ra.sum()) > int(rd.sum())  # the lobe samples are extra intersect() calls


@pytest.mark.gpu
@pytest.mark.parametrize("glossy,seed", [(10, 0x5EED), (4, 7), (2, 0)])
def test_gpu_glossy_matches_oracle(R, O, glossy, seed):
    import variants as V

    s, p = _cornell(R, glossy, seed)
    W, H = 48, 27
    ctx = R.Context(s)
    cam = R.camera_from_trackball(aspect=R.aspect_of(W, H))
    ref, rays = O.Oracle(s).render(p, W, H)
    base = None
    for v in V.all_variants(R):
        with V.options(R, ctx, v):
            img, st = ctx.render(cam, p, W, H)
        assert st.rays == rays, v
        assert float(np.max(np.abs(img - ref))) <= 1e-5, v
        if base is None:
            base = img
        assert img.tobytes() == base.tobytes(), v
    ctx.close()


@pytest.mark.gpu
def test_gpu_glossy_shade_matches_oracle(R, O, golden_dir):
    s, p = _cornell(R, 8, 99)
    z = np.load(f"{golden_dir}/kats.npz")
    rays = z["C5__rays"][:400]
    ctx = R.Context(s)
    rgb, cnt = ctx.shade(rays, p)
    ref, rcnt = O.Oracle(s).shade(rays, p)
    ctx.close()
    assert np.array_equal(cnt, rcnt)
    assert float(np.max(np.abs(rgb - ref))) <= 1e-5
