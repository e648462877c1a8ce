"""GPU parity of the float64 aggregation (flc_weighted_sum_f64, flc_fedopt_step_f64, flc_feddr_combine_f64) against
the reference's own float64 server updates (tests/golden/agg_f64.npz) and the oracle.

The folds are bit-exact (one fp64 fma per element per message, as torch's add_ with alpha); FedAvg's step too.  The
adaptive steps divide by sqrt(v) + tau: torch's CPU sqrt (SLEEF) is not correctly rounded in fp64 either, while the
kernel's is IEEE, so theta is checked within 1e-14 of its update plus one ulp, and v bit for bit.
"""

import numpy as np
import pytest
import torch

from oracle import aggregation_ref as agg_ref
from tests import golden_cases as gc
from tests import golden_f64 as g64
from tests.golden.gen_golden import (CONFIG1_SHAPES, FEDDR_CFG, FEDDR_REGS, SMALL_SHAPES, feddr_inputs, make_model,
                                     make_msgs, scaffold_inputs)


pytestmark = pytest.mark.gpu

AGG = np.load(f"{gc.GOLDEN}/agg_f64.npz", allow_pickle=False)
F64 = torch.float64


def _dev(ts):
    return [t.detach().clone().cuda() for t in ts]


def _msgs_dev(msgs, key):
    return [{**m, key: _dev(m[key])} for m in msgs]


def _flat(ts):
    return torch.cat([t.detach().reshape(-1).cpu() for t in ts]).numpy()


def _golden(key, ts):
    flat = _flat(ts)
    assert flat.dtype == np.float64
    return gc.sha(flat) == str(AGG[key + "|sha"]), flat


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("opt,lr,betas,tau", [("avg", 1, (0, 1), 1), ("adam", 0.01, (0.9, 0.99), 1e-3),
                                               ("yogi", 0.01, (0.9, 0.99), 1e-3), ("adagrad", 0.05, (0.0, 0.99), 1e-3)])
def test_fedopt_update_f64_matches_reference(tag, shapes, opt, lr, betas, tau):
    from fl_sim_amd import aggregation

    params = _dev([p.data for p in make_model(shapes, 1, F64).parameters()])
    g = torch.Generator().manual_seed(2)
    delta = [torch.randn(sh, generator=g, dtype=F64) * 1e-3 for sh in shapes]
    v = None if opt == "avg" else [torch.rand(sh, generator=g, dtype=F64) * 1e-4 + 1e-6 for sh in shapes]
    msgs = make_msgs(shapes, 10, 3, "delta_parameters", F64)
    delta_d, v_d = _dev(delta), (None if v is None else _dev(v))
    aggregation.fedopt_update(params, delta_d, v_d, _msgs_dev(msgs, "delta_parameters"), opt, lr, betas, tau)
    torch.cuda.synchronize()
    assert _golden(f"fedopt_{opt}_{tag}|delta", delta_d)[0], "delta average must be bit-exact"
    ok_theta, got = _golden(f"fedopt_{opt}_{tag}|theta", params)
    if opt == "avg":
        assert ok_theta, "FedAvg must be bit-exact"
        return
    assert _golden(f"fedopt_{opt}_{tag}|v", v_d)[0], "v must be bit-exact"
    p2 = [p.data for p in make_model(shapes, 1, F64).parameters()]
    g = torch.Generator().manual_seed(2)
    d2 = [torch.randn(sh, generator=g, dtype=F64) * 1e-3 for sh in shapes]
    v2 = [torch.rand(sh, generator=g, dtype=F64) * 1e-4 + 1e-6 for sh in shapes]
    agg_ref.fedopt_update(p2, d2, v2, msgs, opt, lr, betas, tau)
    exp_t = _flat(p2)
    theta0 = _flat([p.data for p in make_model(shapes, 1, F64).parameters()])
    assert np.all(np.abs(exp_t - got) <= 1e-14 * np.abs(exp_t - theta0) + np.spacing(np.abs(exp_t)))


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("size_aware", [False, True])
@pytest.mark.parametrize("inertia", [0.0, 0.3])
def test_avg_parameters_f64_matches_reference(tag, shapes, size_aware, inertia):
    from fl_sim_amd import aggregation

    params = _dev([p.data for p in make_model(shapes, 4, F64).parameters()])
    aggregation.avg_parameters(params, _msgs_dev(make_msgs(shapes, 10, 5, "parameters", F64), "parameters"),
                               size_aware, inertia)
    assert _golden(f"avgp_{int(size_aware)}_{inertia}_{tag}|theta", params)[0]


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_update_gradients_f64_matches_reference(tag, shapes):
    from fl_sim_amd import aggregation

    model = make_model(shapes, 6, F64).cuda()
    aggregation.update_gradients(list(model.parameters()), _msgs_dev(make_msgs(shapes, 10, 7, "gradients", F64),
                                                                     "gradients"))
    assert all(p.grad.dtype == F64 for p in model.parameters())
    assert _golden(f"gradients_{tag}|grad", [p.grad for p in model.parameters()])[0]


@pytest.mark.parametrize("n_src", [0, 1, 5, 16, 17, 40])
@pytest.mark.parametrize("n", [1, 7, 1000, 1 << 20])
def test_weighted_sum_f64_chain_is_sequential_fma(n_src, n):
    from fl_sim_amd import codec

    g = torch.Generator().manual_seed(n + n_src)
    srcs = [torch.randn(n, generator=g, dtype=F64) for _ in range(n_src)]
    w = [1.0 / (i + 3) for i in range(n_src)]  # Python doubles, used as given
    dst0 = torch.randn(n, generator=g, dtype=F64)
    exp = dst0.clone().mul_(0.3)
    for s, wi in zip(srcs, w):
        exp.add_(s, alpha=wi)
    dst = dst0.cuda()
    codec.weighted_sum(dst, [s.cuda() for s in srcs], w, init_mode=0, beta=0.3)
    assert g64.same_bits(dst.cpu().numpy(), exp.numpy())


@pytest.mark.parametrize("reg", FEDDR_REGS)
def test_feddr_update_f64_matches_oracle(reg):
    from fl_sim_amd import aggregation

    p, y, xt, msgs = feddr_inputs(SMALL_SHAPES)
    p, y, xt = [t.double() for t in p], [t.double() for t in y], [t.double() for t in xt]
    msgs = [{**m, "x_hat_delta": [t.double() for t in m["x_hat_delta"]]} for m in msgs]
    exp = [[t.clone() for t in ts] for ts in (p, y, xt)]
    cfg = (FEDDR_CFG["alpha"], FEDDR_CFG["eta"], FEDDR_CFG["num_clients"], reg)
    agg_ref.feddr_update(exp[0], exp[1], exp[2], msgs, *cfg)
    got = [_dev(ts) for ts in (p, y, xt)]
    aggregation.feddr_update(got[0], got[1], got[2], _msgs_dev(msgs, "x_hat_delta"), *cfg)
    for e, gt in zip(exp[1:], got[1:]):  # y and x_tilde: bit-exact
        assert g64.same_bits(_flat(gt), _flat(e))
    ge, gg = _flat(exp[0]), _flat(got[0])
    if reg == "l2_norm":  # the norm of the combined theta: an fp64 sum of squares in another order
        np.testing.assert_allclose(gg, ge, rtol=1e-13, atol=0)
    else:
        assert g64.same_bits(gg, ge)


def test_scaffold_update_f64_matches_oracle():
    from fl_sim_amd import aggregation

    shapes = SMALL_SHAPES
    params, cvs, msgs = scaffold_inputs(shapes)
    params, cvs = [t.double() for t in params], [t.double() for t in cvs]
    msgs = [{**m, "parameters_delta": [t.double() for t in m["parameters_delta"]],
             "control_variates_delta": [t.double() for t in m["control_variates_delta"]]} for m in msgs]
    ep, ec = [t.clone() for t in params], [t.clone() for t in cvs]
    agg_ref.scaffold_update(ep, ec, msgs, 0.1, 20)
    gp, gcv = _dev(params), _dev(cvs)
    m_dev = [{**m, "parameters_delta": _dev(m["parameters_delta"]),
              "control_variates_delta": _dev(m["control_variates_delta"])} for m in msgs]
    aggregation.scaffold_update(gp, gcv, m_dev, 0.1, 20)
    assert g64.same_bits(_flat(gp), _flat(ep)) and g64.same_bits(_flat(gcv), _flat(ec))
