"""Host-side check of the view-batch job layout (rt_megakernel.hip: xq_lo / view_job).

The dynamic-fetch kernel hands out jobs from 8 per-XCD ranges; in a batch of V views, range x holds
band x of view 0, then band x of view 1, ...  These loops restate the device integer arithmetic
line for line and check, for ragged and tiny frames, that the ranges tile [0, V * view_jobs)
and that view_job is a bijection onto (view, job) pairs -- every pixel job of every view is
handed out exactly once.  (The GPU tests check the rendered result: test_view_batch_bit_identical.)
"""
import pytest


def xq_lo(n_views, view_jobs, x):
    # J.n_views * (((x * ((J.view_jobs + 63) >> 6)) >> 3) << 6)
    return n_views * (((x * ((view_jobs + 63) >> 6)) >> 3) << 6)


def view_job(n_views, view_jobs, g):
    if n_views <= 1:
        return 0, g
    nt = (view_jobs + 63) >> 6
    x = 7
    while x > 0 and g < n_views * (((x * nt) >> 3) << 6):
        x -= 1
    lo = ((x * nt) >> 3) << 6
    hi = view_jobs if x == 7 else (((x + 1) * nt) >> 3) << 6
    k = g - n_views * lo
    v = k // (hi - lo)
    return v, lo + (k - v * (hi - lo))


def tiles_jobs(W, H, band_rows=8, band_count=1, band_rank=0):
    nbands = (H + band_rows - 1) // band_rows
    n_local = (nbands - band_rank + band_count - 1) // band_count if nbands > band_rank else 0
    return ((W + 7) // 8) * ((band_rows + 7) // 8) * n_local * 64


@pytest.mark.parametrize("W,H,V,count,rank", [(8, 8, 3, 1, 0), (100, 61, 5, 1, 0), (100, 61, 5, 3, 1),
                                              (64, 8, 16, 1, 0), (320, 184, 3, 1, 0), (33, 17, 2, 2, 1),
                                              (256, 136, 1, 1, 0)])
def test_ranges_tile_the_batch_and_decode_is_a_bijection(W, H, V, count, rank):
    vj = tiles_jobs(W, H, 8, count, rank)
    njobs = V * vj
    # ranges: contiguous, ordered, covering [0, njobs) (s_lim of range 7 = J.njobs)
    bounds = [xq_lo(V, vj, x) for x in range(8)] + [njobs]
    assert bounds[0] == 0 and all(a <= b for a, b in zip(bounds, bounds[1:]))
    seen = set()
    for x in range(8):
        for g in range(bounds[x], bounds[x + 1]):
            v, job = view_job(V, vj, g)
            assert 0 <= v < V and 0 <= job < vj
            if V > 1:  # the range of band x holds band x of every view, views in order
                lo = xq_lo(1, vj, x)
                hi = vj if x == 7 else xq_lo(1, vj, x + 1)
                assert lo <= job < hi
            seen.add((v, job))
    assert len(seen) == njobs
