"""Oracle self-consistency (CPU): the O(n) kept-set selection and the indexed Philox stream equal their
reference restatements (the stable argsort of compressors.py:293-296 and philox_uniforms)."""

import numpy as np
import pytest

from oracle import compressors_ref as ref


@pytest.mark.parametrize("n,K", [(10, 3), (1000, 10), (4099, 41), (4099, 4098), (5000, 1)])
def test_topk_kept_select_equals_stable_argsort(n, K):
    g = np.random.default_rng(n * 7 + K)
    for trial in range(25):
        if trial % 2:
            x = g.integers(-3, 4, n).astype(np.float32)  # heavy ties
        else:
            x = (g.standard_normal(n) * 1e-3).astype(np.float32)
        x[g.random(n) < 0.1] = -0.0
        if trial % 3 == 0:
            x[g.random(n) < 0.05] = np.nan
        a, av = ref.topk_kept(x, K)
        b, bv = ref.topk_kept_select(x, K)
        assert np.array_equal(a, b)
        assert np.array_equal(av.view(np.uint32), bv.view(np.uint32))


def test_philox_at_equals_stream():
    u = ref.philox_uniforms(10_007, 5, 9)
    idx = np.random.default_rng(0).integers(0, 10_007, 500)
    assert np.array_equal(ref.philox_uniforms_at(idx, 5, 9), u[idx])
