"""Pin the oracle's float64 forms to the reference's own outputs on float64 vectors (tests/golden/codec_f64.npz).

The reference runs every compressor on whatever dtype x has (compressors.py:267-410); gen_golden.py ``f64`` ran
its Compressor.compressVector on float64 vectors.  Dense cases match bit for bit with the global RNG streams in
lock-step afterwards; top-k satisfies the tie-tolerant rule; the p = 2 norm that underflows to 0 under nonzero
elements raises the reference's IndexError.
"""

import random

import numpy as np
import pytest

from oracle import compressors_ref as ref
from tests import golden_cases as gc
from tests import golden_f64 as g64

F64 = g64.load()
ADAPTIVE = {k: v for k, v in F64.items() if k.startswith("adaptive")}
DENSE = {k: v for k, v in F64.items() if k.split("|")[0] not in ("topk", "randk") and k not in ADAPTIVE}
SPARSE = {k: v for k, v in F64.items() if k.split("|")[0] in ("topk", "randk")}


@pytest.mark.parametrize("case", sorted(DENSE))
def test_f64_dense_oracle_matches_reference(case):
    rec = DENSE[case]
    name, _, seed = case.split("|")
    x = g64.case_input(case, rec)
    assert x.dtype == np.float64
    gc.seed_all(int(seed))
    if "error" in rec:
        with pytest.raises(IndexError) as ei:
            g64.oracle_dense(name, x)
        assert str(rec["error"]).endswith(str(ei.value))
        return
    out, send = g64.oracle_dense(name, x)
    assert out.dtype == np.float64
    assert g64.check_output(rec, out), case
    assert float(send) == float(rec["send"]), (send, rec["send"])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


@pytest.mark.parametrize("case", sorted(SPARSE))
def test_f64_sparse_oracle_matches_reference(case):
    rec = SPARSE[case]
    parts = case.split("|")
    name, K, seed = parts[0], int(parts[2]), int(parts[-1])
    x = g64.case_input(case, rec)
    gc.seed_all(seed)
    out, send = gc.oracle_sparse(name, x, len(x), K)
    assert out.dtype == np.float64
    if name == "topk":
        assert g64.topk_valid(x, out, K), case
        if "out" in rec:
            assert g64.topk_valid(x, rec["out"], K)
    else:
        assert g64.check_output(rec, out), case
    assert float(send) == float(rec["send"])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])


@pytest.mark.parametrize("case", sorted(ADAPTIVE))
def test_f64_adaptive_oracle_matches_reference(case):
    rec = ADAPTIVE[case]
    x = g64.case_input(case, rec)
    gc.seed_all(int(case.split("|")[-1]))
    if "error" in rec:
        with np.errstate(all="ignore"):
            p = np.abs(x) / np.abs(x).sum()
        # numpy's checks before the draw (mtrand choice): NaN, then |sum - 1| > sqrt(eps64)
        err = "probabilities contain NaN" if np.isnan(p.sum()) else (
            "probabilities do not sum to 1" if abs(p.sum() - 1.0) > np.sqrt(np.finfo(np.float64).eps) else "")
        assert err == str(rec["error"])
        return
    out, send, ind = ref.adaptive_random(x, len(x), np.random.random_sample())
    assert out.dtype == np.float64
    assert [ind] == list(rec["index"])
    assert g64.check_output(rec, out), case
    assert random.random() == float(rec["next_random"])


def test_f64_fixture_covers_every_compressor_type():
    names = {k.split("|")[0] for k in F64}
    for want in ("identical", "lazy_p03", "natural64", "natural32", "stddither64_s8_p2", "natdither64_s3_p2",
                 "stddither32_s8_inf", "topk", "randk", "adaptive", "adaptive_heavy", "adaptive_err"):
        assert want in names, want
    assert any("error" in rec for rec in F64.values()), "the underflowed-norm IndexError case"


def test_natural64_power_of_two_maps_to_itself():
    x = np.array([2.0**-1074, 2.0**-1000, 0.5, 1.0, 2.0**1000, -(2.0**300)])
    out, _, _ = ref.natural64(x, lambda idx: np.zeros(len(idx)))
    assert np.array_equal(out, x)
