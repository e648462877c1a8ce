"""The CPU-PyTorch baseline path (oracle/torch_ref.py, bench.py cpu_baseline) computes the stacked codec:
the same kept set as the oracle and decoded values within one level step of the input."""

import numpy as np
import torch

from oracle import compressors_ref as ref
from oracle import torch_ref


def test_torch_stacked_matches_oracle_semantics():
    n, k, s = 100_003, 1000, 127
    x = (np.random.default_rng(0).standard_normal(n) * 1e-3).astype(np.float32)
    out = torch_ref.stacked_step(torch.from_numpy(x), k, s, torch.Generator().manual_seed(1)).numpy()
    kept, vals = ref.topk_kept_select(x, k)
    nz = np.flatnonzero(out)
    assert set(nz) <= set(kept)
    norm = np.abs(vals).max()
    assert np.all(np.abs(out[kept] - x[kept]) <= norm / s * (1 + 1e-6))
    assert np.all(out[np.setdiff1d(np.arange(n), kept)] == 0)
    assert np.all(np.sign(out[nz]) == np.sign(x[nz]))
