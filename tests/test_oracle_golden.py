"""Pin the oracle (oracle/compressors_ref.py, oracle/aggregation_ref.py) to the reference's own outputs.

The fixtures in tests/golden/ were produced by running wenh06/fl-sim's Compressor.compressVector and
its aggregation method bodies (gen_golden.py).  Every dense codec case must match bit for bit with the
global RNG streams in lock-step afterwards; top-k must satisfy the tie-tolerant rule (the reference's
argsort is unstable) and match exactly wherever the K-th largest value is unique.
"""

import random

import numpy as np
import pytest
import torch

from oracle import aggregation_ref as agg_ref
from oracle import compressors_ref as ref
from tests import golden_cases as gc

DENSE = gc.load("codec_dense.npz")
SPARSE = gc.load("codec_sparse.npz")
AGG = np.load(f"{gc.GOLDEN}/agg.npz", allow_pickle=False)


def topk_valid(x, out, K):
    return gc.topk_valid(x, out, K)


@pytest.mark.parametrize("case", sorted(DENSE))
def test_dense_codec_matches_reference(case):
    rec = DENSE[case]
    name, _, seed = case.split("|")
    x = gc.case_input(case, rec)
    gc.seed_all(int(seed))
    out, send = gc.oracle_dense(name, x)
    assert gc.check_output(case, rec, out), case
    assert float(send) == float(rec["send"]), (send, rec["send"])
    # the global streams advanced exactly as the reference advanced them
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


@pytest.mark.parametrize("case", sorted(SPARSE))
def test_sparse_codec_matches_reference(case):
    rec = SPARSE[case]
    parts = case.split("|")
    name, seed = parts[0], int(parts[-1])
    x = gc.case_input(case, rec)
    if name == "adaptive":
        D, K = len(x), 1
    else:
        D = len(x)
        K = int(parts[2])
        if name == "randk":
            K = max(K, 1)
    gc.seed_all(seed)
    out, send = gc.oracle_sparse(name, x, D, K)
    if name == "topk":
        assert topk_valid(x, out, K), case
        if "out" in rec:
            assert topk_valid(x, rec["out"], K), "fixture itself violates the rule?"
            t = ref.topk_threshold(x, K) if 0 < K < len(x) else None
            if t is None or np.sum(x == t) == 1:
                assert gc.same_bits(out, rec["out"]), case
        else:
            assert gc.check_output(case, rec, out)
    else:
        assert gc.check_output(case, rec, out), case
    assert float(send) == float(rec["send"])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


# ------------------------------------------------------------------------------------------ aggregation
from tests.golden.gen_golden import CONFIG1_SHAPES, SMALL_SHAPES, make_model, make_msgs  # noqa: E402


def _flat(ts):
    return torch.cat([t.detach().reshape(-1) for t in ts]).numpy()


def _check(key, ts):
    flat = _flat(ts)
    if key + "|out" in AGG.files:
        assert gc.same_bits(flat, AGG[key + "|out"]), key
    assert gc.sha(flat) == str(AGG[key + "|sha"]), key


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("opt,lr,betas,tau", [("avg", 1, (0, 1), 1), ("adam", 0.01, (0.9, 0.99), 1e-3),
                                               ("yogi", 0.01, (0.9, 0.99), 1e-3), ("adagrad", 0.05, (0.0, 0.99), 1e-3)])
def test_fedopt_oracle_matches_reference(tag, shapes, opt, lr, betas, tau):
    torch.set_num_threads(1)
    model = make_model(shapes, 1)
    params = [p.data for p in model.parameters()]
    g = torch.Generator().manual_seed(2)
    delta = [torch.randn(sh, generator=g) * 1e-3 for sh in shapes]
    v = None if opt == "avg" else [torch.rand(sh, generator=g) * 1e-4 + 1e-6 for sh in shapes]
    msgs = make_msgs(shapes, 10, 3, "delta_parameters")
    agg_ref.fedopt_update(params, delta, v, msgs, opt, lr, betas, tau)
    _check(f"fedopt_{opt}_{tag}|theta", params)
    _check(f"fedopt_{opt}_{tag}|delta", delta)
    if v is not None:
        _check(f"fedopt_{opt}_{tag}|v", v)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("size_aware", [False, True])
@pytest.mark.parametrize("inertia", [0.0, 0.3])
def test_avg_parameters_oracle_matches_reference(tag, shapes, size_aware, inertia):
    model = make_model(shapes, 4)
    params = [p.data for p in model.parameters()]
    agg_ref.avg_parameters(params, make_msgs(shapes, 10, 5, "parameters"), size_aware, inertia)
    _check(f"avgp_{int(size_aware)}_{inertia}_{tag}|theta", params)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_update_gradients_oracle_matches_reference(tag, shapes):
    grads = agg_ref.update_gradients(None, make_msgs(shapes, 10, 7, "gradients"))
    _check(f"gradients_{tag}|grad", grads)


def test_philox_oracle_known_answer():
    # Random123 known-answer vector for philox4x32_10(ctr=0, key=0)
    c = ref.philox4x32_10([0], [0], [0], [0], np.uint32(0), np.uint32(0))
    assert [int(v[0]) for v in c] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    c = ref.philox4x32_10([0xFFFFFFFF], [0xFFFFFFFF], [0xFFFFFFFF], [0xFFFFFFFF], np.uint32(0xFFFFFFFF),
                          np.uint32(0xFFFFFFFF))
    assert [int(v[0]) for v in c] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


# ------------------------------------------------------------------- aggregation variants
from tests.golden.gen_golden import (  # noqa: E402
    FEDDR_CFG, FEDDR_REGS, SCAFFOLD_CFG, feddr_inputs, ifca_inputs, scaffold_inputs)

AGGV = np.load(f"{gc.GOLDEN}/agg_variants.npz", allow_pickle=False)


def _check_v(key, ts):
    flat = _flat(ts)
    if key + "|out" in AGGV.files:
        assert gc.same_bits(flat, AGGV[key + "|out"]), key
    assert gc.sha(flat) == str(AGGV[key + "|sha"]), key


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_scaffold_oracle_matches_reference(tag, shapes):
    params, cvs, msgs = scaffold_inputs(shapes)
    agg_ref.scaffold_update(params, cvs, msgs, SCAFFOLD_CFG["lr"], SCAFFOLD_CFG["num_clients"])
    _check_v(f"scaffold_{tag}|theta", params)
    _check_v(f"scaffold_{tag}|cv", cvs)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_ifca_oracle_matches_reference(tag, shapes):
    centers, msgs = ifca_inputs(shapes)
    agg_ref.ifca_update(centers, msgs, 4)
    for c in range(4):
        _check_v(f"ifca_{tag}|center{c}", centers[c]["center_model_params"])
        assert centers[c]["client_ids"] == AGGV[f"ifca_{tag}|ids{c}"].tolist()


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("reg", FEDDR_REGS)
def test_feddr_oracle_matches_reference(tag, shapes, reg):
    torch.set_num_threads(1)  # the l2 prox's norm is a torch CPU sum, as when the fixtures were made
    params, ys, xts, msgs = feddr_inputs(shapes)
    agg_ref.feddr_update(params, ys, xts, msgs, FEDDR_CFG["alpha"], FEDDR_CFG["eta"], FEDDR_CFG["num_clients"], reg)
    _check_v(f"feddr_{reg}_{tag}|theta", params)
    _check_v(f"feddr_{reg}_{tag}|y", ys)
    _check_v(f"feddr_{reg}_{tag}|xtil", xts)


def test_feddr_linf_raises_like_reference():
    params, ys, xts, msgs = feddr_inputs(SMALL_SHAPES)
    with pytest.raises(NotImplementedError):
        agg_ref.feddr_update(params, ys, xts, msgs, 0.9, 0.05, 10, "linf_norm")


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_client_delta_oracle_matches_reference(tag, shapes):
    from tests.golden.gen_golden import delta_inputs

    local, cached = delta_inputs(shapes)
    _check_v(f"delta_{tag}|delta", agg_ref.client_delta(local, cached))


# ------------------------------------------------------------------- FedDyn / pFedMe server updates (round 5)
from tests.golden.gen_golden import FEDDYN_CFG, PFEDME_BETAS, feddyn_inputs, pfedme_inputs  # noqa: E402


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("nm", [10, 20, 0])
def test_feddyn_oracle_matches_reference(tag, shapes, nm):
    params, hs, msgs = feddyn_inputs(shapes, nm)
    agg_ref.feddyn_update(params, hs, msgs, FEDDYN_CFG["mu"], FEDDYN_CFG["num_clients"])
    _check_v(f"feddyn_{nm}_{tag}|theta", params)
    _check_v(f"feddyn_{nm}_{tag}|h", hs)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("nm", [10, 20, 0])
@pytest.mark.parametrize("beta", PFEDME_BETAS)
def test_pfedme_oracle_matches_reference(tag, shapes, nm, beta):
    params, msgs = pfedme_inputs(shapes, nm)
    agg_ref.pfedme_update(params, msgs, beta)
    _check_v(f"pfedme_{beta}_{nm}_{tag}|theta", params)
