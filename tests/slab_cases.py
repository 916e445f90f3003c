"""Box / ray pairs for the slab-test bound checks (tests/test_gpu_slab.py on the device, tests/test_slab_bounds.py
as a numpy restatement): random pairs and the pairs that stress the quotient bounds."""
import numpy as np


def unit(v):
    v = np.asarray(v, np.float32)
    return (v / np.linalg.norm(v.astype(np.float64), axis=-1, keepdims=True)).astype(np.float32)


def pairs(rng, n):
    boxes, rays = [], []
    # random boxes and rays
    c = rng.uniform(-2, 2, (n, 3)).astype(np.float32)
    h = rng.uniform(0.01, 1, (n, 3)).astype(np.float32)
    boxes.append(np.concatenate([c - h, c + h], 1))
    o = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    aim = c + h * rng.uniform(-1.5, 1.5, (n, 3)).astype(np.float32)  # about half of them hit
    rays.append(np.concatenate([o, unit(aim - o)], 1))
    # grazing: rays aimed at a box corner or an edge point, origin a few ulps off the exact line
    lo = (c - h).astype(np.float32)
    hi = (c + h).astype(np.float32)
    sel = rng.integers(0, 2, (n, 3)).astype(bool)
    corner = np.where(sel, lo, hi)
    edge = corner.copy()
    ax = rng.integers(0, 3, n)
    edge[np.arange(n), ax] = rng.uniform(lo[np.arange(n), ax], hi[np.arange(n), ax]).astype(np.float32)
    for target in (corner, edge):
        d = unit(rng.normal(size=(n, 3)))
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
    rays.append(np.concatenate([o, unit(d)], 1))
    # axis-parallel and near-axis-parallel directions (tiny and zero components: the IEEE path)
    d = np.zeros((n, 3), np.float32)
    d[np.arange(n), rng.integers(0, 3, n)] = 1.0
    d += rng.choice([0.0, 1e-30, 1e-13, 1e-7, 1e-3], (n, 3)).astype(np.float32) * rng.choice([-1, 1], (n, 3))
    boxes.append(np.concatenate([lo, hi], 1))
    rays.append(np.concatenate([rng.uniform(-4, 4, (n, 3)).astype(np.float32), unit(d)], 1))
    # far boxes and degenerate (flat) boxes
    far = rng.uniform(-1e13, 1e13, (n, 3)).astype(np.float32)
    flat = np.concatenate([lo, hi], 1)
    flat[:, 3 + ax % 3] = flat[:, ax % 3]
    boxes.append(np.concatenate([far, far + 1.0], 1))
    rays.append(np.concatenate([np.zeros((n, 3), np.float32), unit(far + 0.5)], 1))
    boxes.append(flat)
    rays.append(np.concatenate([rng.uniform(-4, 4, (n, 3)).astype(np.float32), unit(rng.normal(size=(n, 3)))], 1))
    return np.concatenate(boxes).astype(np.float32), np.concatenate(rays).astype(np.float32)
