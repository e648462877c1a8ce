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


def test_torch_dither_topk_and_round_semantics():
    g = torch.Generator().manual_seed(2)
    X = torch.randn(3, 5001, generator=g) * 1e-3
    X[:, ::11] = 0
    out = torch_ref.dither_step(X, 127, g)
    norm = X.abs().amax(dim=1, keepdim=True)
    assert torch.all((out - X).abs() <= norm / 127 * (1 + 1e-6))
    assert torch.all(out[X == 0] == 0) and torch.all(torch.sign(out[out != 0]) == torch.sign(X[out != 0]))
    x = X[0].clone()
    t = torch_ref.topk_step(x, 50)
    kept, vals = ref.topk_kept_select(x.numpy(), 50)
    assert np.count_nonzero(t.numpy()) == 50 and set(np.flatnonzero(t.numpy())) <= set(kept) | set(np.flatnonzero(x.numpy() == vals.min()))
    r = torch_ref.round_fold([X[0], X[1]], [0.25, 0.75], 50, 127, g)
    assert r.shape == X[0].shape and np.count_nonzero(r.numpy()) <= 100
