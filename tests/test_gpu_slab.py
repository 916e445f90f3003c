"""The kernels' reference slab test (src/ray_tracing.cpp:213-264) decided from bounds on its quotients
(rt_kernels.hip ref_slab_bounds, RT_SLAB_FILTER): wherever the bounds give an answer it must be the answer of
the reference's IEEE quotients (ref_slab_div), on random pairs and on the pairs that stress the bounds --
grazing rays through box edges and corners (tin == tout up to an ulp), origins on a box plane (zero
numerators), axis-parallel and near-axis-parallel directions, far boxes.  The candidate culling the images
depend on runs through this test, so the image parity tests cover it too; this one aims at the ties."""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "raytracer-group27_amd"))
import rt_amd as R  # noqa: E402

pytestmark = pytest.mark.gpu


def _unit(v):
    v = np.asarray(v, np.float32)
    return (v / np.linalg.norm(v.astype(np.float64), axis=-1, keepdims=True)).astype(np.float32)


def _pairs(rng, n):
    boxes, rays = [], []
    # random boxes and rays
    c = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    h = rng.uniform(0.01, 1, (n, 3)).astype(np.float32)
    boxes.append(np.concatenate([c - h, c + h], 1))
    rays.append(np.concatenate([rng.uniform(-4, 4, (n, 3)).astype(np.float32), _unit(rng.normal(size=(n, 3)))], 1))
    # grazing: rays aimed at a box corner or an edge point, origin a few ulps off the exact line
    lo = (c - h).astype(np.float32)
    hi = (c + h).astype(np.float32)
    sel = rng.integers(0, 2, (n, 3)).astype(bool)
    corner = np.where(sel, lo, hi)
    edge = corner.copy()
    ax = rng.integers(0, 3, n)
    edge[np.arange(n), ax] = rng.uniform(lo[np.arange(n), ax], hi[np.arange(n), ax]).astype(np.float32)
    for target in (corner, edge):
        d = _unit(rng.normal(size=(n, 3)))
        t = rng.uniform(0.1, 5, (n, 1)).astype(np.float32)
        o = (target - t * d).astype(np.float32)
        ulps = rng.integers(-3, 4, (n, 3)).astype(np.int32)
        o = (o.view(np.int32) + ulps).view(np.float32)
        boxes.append(np.concatenate([lo, hi], 1))
        rays.append(np.concatenate([o, d], 1))
    # origins on a box plane (exact zero numerators), some directions along the box face
    o = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    k = rng.integers(0, 3, n)
    o[np.arange(n), k] = np.where(rng.integers(0, 2, n) == 1, lo[np.arange(n), k], hi[np.arange(n), k])
    d = rng.normal(size=(n, 3))
    d[np.arange(n), k] *= rng.integers(0, 2, n)  # half of them parallel to that plane
    boxes.append(np.concatenate([lo, hi], 1))
    rays.append(np.concatenate([o, _unit(d)], 1))
    # axis-parallel and near-axis-parallel directions (tiny and zero components: the IEEE path)
    d = np.zeros((n, 3), np.float32)
    d[np.arange(n), rng.integers(0, 3, n)] = 1.0
    d += rng.choice([0.0, 1e-30, 1e-13, 1e-7, 1e-3], (n, 3)).astype(np.float32) * rng.choice([-1, 1], (n, 3))
    boxes.append(np.concatenate([lo, hi], 1))
    rays.append(np.concatenate([rng.uniform(-4, 4, (n, 3)).astype(np.float32), _unit(d)], 1))
    # far boxes and degenerate (flat) boxes
    far = rng.uniform(-1e13, 1e13, (n, 3)).astype(np.float32)
    flat = np.concatenate([lo, hi], 1)
    flat[:, 3 + ax % 3] = flat[:, ax % 3]
    boxes.append(np.concatenate([far, far + 1.0], 1))
    rays.append(np.concatenate([np.zeros((n, 3), np.float32), _unit(far + 0.5)], 1))
    boxes.append(flat)
    rays.append(np.concatenate([rng.uniform(-4, 4, (n, 3)).astype(np.float32), _unit(rng.normal(size=(n, 3)))], 1))
    return np.concatenate(boxes).astype(np.float32), np.concatenate(rays).astype(np.float32)


def test_slab_bounds_agree_with_ieee_quotients():
    rng = np.random.default_rng(2026)
    boxes, rays = _pairs(rng, 200000)
    out = R.slab_check(boxes, rays)
    exact, bound = out & 1, out >> 1
    assert set(np.unique(bound)) <= {0, 1, 2}
    decided = bound != 2
    bad = np.nonzero(decided & (bound != exact))[0]
    assert len(bad) == 0, (len(bad), boxes[bad[:4]].tolist(), rays[bad[:4]].tolist())
    n = 200000
    random_open = float(np.mean(bound[:n] == 2))
    grazing_open = float(np.mean(bound[n:3 * n] == 2))
    print(f"open: random {random_open:.5f}, grazing {grazing_open:.4f}, all {float(np.mean(~decided)):.4f}; "
          f"hits {float(np.mean(exact)):.3f}")
    assert random_open < 0.01  # the bounds decide nearly every ordinary pair
    assert exact[n:3 * n].mean() > 0.05 and exact[n:3 * n].mean() < 0.95  # the grazing set straddles the edges
