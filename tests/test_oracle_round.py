"""Pin the compressed-round oracle (oracle/round_ref.py) to the reference's own round (tests/golden/round_codec.npz,
gen_golden.py ``gen_round``: FedOptClient.communicate -> Compressor.compressVector -> FedOptServer.update, run from
the reference's sources): the server's θ, δ and v bit for bit, every client's send statistics, and both global
streams in lock-step after the round.  CPU only."""

import random

import numpy as np
import pytest
import torch

from oracle import round_ref
from tests import golden_cases as gc
from tests.golden.gen_golden import (CONFIG1_SHAPES, ROUND_CODECS, ROUND_OPTS, SMALL_SHAPES, round_inputs,
                                     round_seed)

ROUND = gc.load("round_codec.npz")


def flat(ts):
    return torch.cat([t.detach().reshape(-1) for t in ts]).numpy()


def check(rec, field, ts):
    a = flat(ts)
    if "out" in rec.get(field, {}):
        return gc.same_bits(a, rec[field]["out"])
    return gc.sha(a) == str(rec[field]["sha"])


def fields(case):
    """{field: {"sha": ..., "out": ...}} of one round case (keys ``round_<codec>_<opt>_<tag>|<field>|sha``)."""
    out = {}
    for k, v in ROUND.items():
        if k.startswith(case + "|"):
            out.setdefault(k.split("|")[1], {})
    z = np.load(f"{gc.GOLDEN}/round_codec.npz", allow_pickle=False)
    for k in z.files:
        parts = k.split("|")
        if parts[0] == case and len(parts) == 3:
            out.setdefault(parts[1], {})[parts[2]] = z[k]
        elif parts[0] == case and len(parts) == 2:
            out[parts[1]] = z[k]
    return out


@pytest.mark.parametrize("tag", ["small", "config1"])
@pytest.mark.parametrize("opt", list(ROUND_OPTS))
@pytest.mark.parametrize("codec", ROUND_CODECS)
def test_round_oracle_matches_reference(codec, opt, tag):
    shapes = SMALL_SHAPES if tag == "small" else CONFIG1_SHAPES
    rec = fields(f"round_{codec}_{opt}_{tag}")
    theta, delta, v, locals_, sizes = round_inputs(shapes, opt)
    cfg = ROUND_OPTS[opt]
    gc.seed_all(round_seed(codec, opt, tag))
    stats = round_ref.fedopt_round(codec, theta, delta, v, locals_, sizes, opt, cfg["lr"], cfg["betas"], cfg["tau"])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])
    assert np.array_equal(np.array(stats, dtype=np.float64), rec["stats"])
    assert check(rec, "theta", theta)
    assert check(rec, "delta", delta)
    if v is not None:
        assert check(rec, "v", v)


VRG = np.load(f"{gc.GOLDEN}/agg_vr.npz", allow_pickle=False)


@pytest.mark.parametrize("tag", ["small", "config1"])
@pytest.mark.parametrize("nm", [10, 20])
@pytest.mark.parametrize("vr", [True, False])
@pytest.mark.parametrize("name", ["fedprox", "fedpd", "proxskip", "pfedmac"])
def test_vr_oracle_matches_reference(name, vr, nm, tag):
    """agg_vr.npz (the reference's FedProx / FedPD / ProxSkip / pFedMac update) through the oracle's avg_parameters and
    update_gradients."""
    from oracle import aggregation_ref as agg_ref
    from tests.golden.gen_golden import PFEDMAC_BETA, vr_inputs

    shapes = SMALL_SHAPES if tag == "small" else CONFIG1_SHAPES
    params, msgs = vr_inputs(shapes, nm)
    agg_ref.avg_parameters(params, msgs, inertia=1 - PFEDMAC_BETA if name == "pfedmac" else 0.0)
    key = f"vr_{name}_{int(vr)}_{nm}_{tag}"

    def same(field, ts):
        a = flat(ts)
        if f"{key}|{field}|out" in VRG.files:
            return gc.same_bits(a, VRG[f"{key}|{field}|out"])
        return gc.sha(a) == str(VRG[f"{key}|{field}|sha"])

    assert same("theta", params)
    if vr:
        assert same("grad", agg_ref.update_gradients(params, msgs))
