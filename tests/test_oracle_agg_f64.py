"""Pin the aggregation oracle on float64 models and messages (tests/golden/agg_f64.npz: the reference's own
FedOptServer.update / avg_parameters / update_gradients run on float64 tensors, gen_golden.py ``agg64``)."""

import numpy as np
import pytest
import torch

from oracle import aggregation_ref as agg_ref
from tests import golden_cases as gc
from tests import golden_f64 as g64
from tests.golden.gen_golden import CONFIG1_SHAPES, SMALL_SHAPES, make_model, make_msgs

AGG = np.load(f"{gc.GOLDEN}/agg_f64.npz", allow_pickle=False)
F64 = torch.float64


def _check(key, ts):
    flat = torch.cat([t.detach().reshape(-1) for t in ts]).numpy()
    assert flat.dtype == np.float64
    if key + "|out" in AGG.files:
        assert g64.same_bits(flat, AGG[key + "|out"]), key
    assert gc.sha(flat) == str(AGG[key + "|sha"]), key


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("opt,lr,betas,tau", [("avg", 1, (0, 1), 1), ("adam", 0.01, (0.9, 0.99), 1e-3),
                                               ("yogi", 0.01, (0.9, 0.99), 1e-3), ("adagrad", 0.05, (0.0, 0.99), 1e-3)])
def test_fedopt_oracle_matches_reference_f64(tag, shapes, opt, lr, betas, tau):
    torch.set_num_threads(1)
    params = [p.data for p in make_model(shapes, 1, F64).parameters()]
    g = torch.Generator().manual_seed(2)
    delta = [torch.randn(sh, generator=g, dtype=F64) * 1e-3 for sh in shapes]
    v = None if opt == "avg" else [torch.rand(sh, generator=g, dtype=F64) * 1e-4 + 1e-6 for sh in shapes]
    agg_ref.fedopt_update(params, delta, v, make_msgs(shapes, 10, 3, "delta_parameters", F64), opt, lr, betas, tau)
    _check(f"fedopt_{opt}_{tag}|theta", params)
    _check(f"fedopt_{opt}_{tag}|delta", delta)
    if v is not None:
        _check(f"fedopt_{opt}_{tag}|v", v)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("size_aware", [False, True])
@pytest.mark.parametrize("inertia", [0.0, 0.3])
def test_avg_parameters_oracle_matches_reference_f64(tag, shapes, size_aware, inertia):
    params = [p.data for p in make_model(shapes, 4, F64).parameters()]
    agg_ref.avg_parameters(params, make_msgs(shapes, 10, 5, "parameters", F64), size_aware, inertia)
    _check(f"avgp_{int(size_aware)}_{inertia}_{tag}|theta", params)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_update_gradients_oracle_matches_reference_f64(tag, shapes):
    _check(f"gradients_{tag}|grad", agg_ref.update_gradients(None, make_msgs(shapes, 10, 7, "gradients", F64)))
