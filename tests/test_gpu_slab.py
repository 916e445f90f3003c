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
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import rt_amd as R  # noqa: E402
from slab_cases import pairs  # noqa: E402

pytestmark = pytest.mark.gpu


def test_slab_bounds_agree_with_ieee_quotients():
    rng = np.random.default_rng(2026)
    boxes, rays = pairs(rng, 200000)
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
