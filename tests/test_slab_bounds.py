"""The quotient bounds of the kernels' slab test (rt_kernels.hip ref_slab_bounds, RT_SLAB_FILTER) restated in
numpy float32 and checked against the reference's IEEE quotients (src/ray_tracing.cpp:220-260, numpy's float32
division is correctly rounded as the reference's): every answer the bounds give must be the quotients' answer.
The device's v_rcp_f32 is within 1 ulp of 1/d; the restatement takes the correctly rounded reciprocal and its
neighbours one ulp either side, so the check covers every reciprocal the hardware may return.  The device
kernel itself is checked the same way by tests/test_gpu_slab.py."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from slab_cases import pairs  # noqa: E402

F = np.float32


def ieee_answer(b, r):
    """ref_slab_div: the reference's quotients, std::min / std::max / glm::max / glm::min and the final test."""
    o, nd = r[:, :3], r[:, 3:]
    with np.errstate(divide="ignore", invalid="ignore"):
        tmin = (b[:, :3] - o) / nd
        tmax = (b[:, 3:] - o) / nd
    tin_k = np.where(tmax < tmin, tmax, tmin)
    tout_k = np.where(tmin < tmax, tmax, tmin)
    tin = tin_k[:, 0]
    tout = tout_k[:, 0]
    for k in (1, 2):
        tin = np.where(tin < tin_k[:, k], tin_k[:, k], tin)
        tout = np.where(tout_k[:, k] < tout, tout_k[:, k], tout)
    return ~((tin > tout) | (tout < 0))


def bound_answer(b, r, rcp_ulps):
    """ref_slab_bounds with the reciprocal moved rcp_ulps (-1, 0, 1) ulps from 1/d: 0 miss, 1 hit, 2 open."""
    o, nd = r[:, :3], r[:, 3:]
    a = np.concatenate([b[:, :3] - o, b[:, 3:] - o], 1)  # lo x y z, hi x y z
    mag_d = nd.view(np.uint32) & np.uint32(0x7FFFFFFF)
    mag_a = a.view(np.uint32) & np.uint32(0x7FFFFFFF)
    LO, HI = np.uint32(0x2B800000), np.uint32(0x53800000)
    ok = ((mag_d.max(1) <= HI) & (mag_d.min(1) >= LO) & (mag_a.max(1) <= HI) &
          ((mag_a - np.uint32(1)).min(1) >= LO - np.uint32(1)))
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        rc = F(1.0) / nd
        if rcp_ulps:
            rc = np.nextafter(rc, np.where(rcp_ulps > 0, F(np.inf), F(-np.inf)).astype(F)).astype(F)
        p0, p1 = a[:, :3] * rc, a[:, 3:] * rc
        qi, qo = np.minimum(p0, p1), np.maximum(p0, p1)
        ei, eo = np.abs(qi) * F(2.0 ** -18), np.abs(qo) * F(2.0 ** -18)
        in_lo, in_hi = (qi - ei).max(axis=1), (qi + ei).max(axis=1)
        out_lo, out_hi = (qo - eo).min(axis=1), (qo + eo).min(axis=1)
        out_neg = qo.min(axis=1) < 0
    ans = np.where(in_lo > out_hi, 0, np.where(~(in_hi <= out_lo), 2, np.where(out_neg, 0, 1)))
    return np.where(ok, ans, 2)


def test_bounds_decide_as_the_ieee_quotients():
    rng = np.random.default_rng(7)
    b, r = pairs(rng, 40000)
    exact = ieee_answer(b, r)
    for u in (-1, 0, 1):
        ans = bound_answer(b, r, u)
        decided = ans != 2
        bad = np.nonzero(decided & (ans != exact.astype(int)))[0]
        assert len(bad) == 0, (u, len(bad), b[bad[:3]].tolist(), r[bad[:3]].tolist())
        assert np.mean(ans[:40000] == 2) < 0.01  # ordinary pairs are decided by the bounds
    # the grazing pairs straddle box edges and corners: both answers occur and some are left open
    graze = exact[40000:120000]
    assert 0.05 < graze.mean() < 0.95
