"""The aggregation drop-in on the reference's own placement: the server model and its optimizer state in HOST memory
(``Server.__init__`` sets ``self.device = torch.device("cpu")``, nodes.py:606), the client messages on a HIP device
(clients on ``cuda:i mod N``, nodes.py:706-713) or in host memory.  The mixins stage the server's tensors, fold on the
device and write the results back into the same host tensors in place; every result must equal the reference's
(tests/golden/agg.npz, agg_variants.npz) bit for bit, exactly as the device-resident server does."""

import numpy as np
import pytest
import torch

from oracle import aggregation_ref as agg_ref
from tests import golden_cases as gc
from tests.golden.gen_golden import (CONFIG1_SHAPES, FEDDR_CFG, SCAFFOLD_CFG, SMALL_SHAPES, feddr_inputs,
                                     ifca_inputs, make_model, make_msgs, scaffold_inputs)

pytestmark = pytest.mark.gpu

AGG = np.load(f"{gc.GOLDEN}/agg.npz", allow_pickle=False)
AGGV = np.load(f"{gc.GOLDEN}/agg_variants.npz", allow_pickle=False)
OPTS = [("avg", 1, (0, 1), 1), ("adam", 0.01, (0.9, 0.99), 1e-3), ("yogi", 0.01, (0.9, 0.99), 1e-3),
        ("adagrad", 0.05, (0.0, 0.99), 1e-3)]


def _flat(ts):
    return torch.cat([t.detach().reshape(-1).cpu() for t in ts]).numpy()


def _sha(ts):
    return gc.sha(_flat(ts))


def _msgs_on(msgs, key, where):
    if where == "host":
        return msgs
    return [{**m, key: [t.to(where) for t in m[key]]} for m in msgs]


@pytest.fixture(autouse=True, params=["zero_copy", "copy"])
def staging_mode(request, monkeypatch):
    """Every test under both stagings of an adopted server: the kernels on the pinned host buffer itself (zero-copy,
    the default) and one copy each way through a device buffer (FLC_HOST_ZEROCOPY=0)."""
    from fl_sim_amd import hoststage

    monkeypatch.setenv("FLC_HOST_ZEROCOPY", "1" if request.param == "zero_copy" else "0")
    hoststage._MIRRORS.clear()
    yield request.param
    hoststage._MIRRORS.clear()


class _Cfg:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _server_cls():
    """A stand-in for the reference's FedOptServer / Server: only the attributes the mixins read, the model on the
    CPU as nodes.py:606 puts it."""
    from fl_sim_amd.aggregation import AggregationMixin, FedOptUpdateMixin

    class Server(FedOptUpdateMixin, AggregationMixin):
        device = torch.device("cpu")

    return Server


def _fedopt_server(shapes, opt, lr, betas, tau, msgs):
    s = _server_cls()()
    s.model = make_model(shapes, 1)
    s.config = _Cfg(optimizer=opt, lr=lr, betas=betas, tau=tau)
    g = torch.Generator().manual_seed(2)
    s.delta_parameters = [torch.randn(sh, generator=g) * 1e-3 for sh in shapes]
    s.v_parameters = None if opt == "avg" else [torch.rand(sh, generator=g) * 1e-4 + 1e-6 for sh in shapes]
    s._received_messages = msgs
    return s


def _check_adaptive_theta(shapes, opt, lr, betas, tau, msgs, got_theta):
    """The adaptive tails vs the oracle (torch CPU): 1e-6 of the update + 1 ulp (torch's CPU sqrt is SLEEF's)."""
    p2 = [p.data for p in make_model(shapes, 1).parameters()]
    g = torch.Generator().manual_seed(2)
    d2 = [torch.randn(sh, generator=g) * 1e-3 for sh in shapes]
    v2 = [torch.rand(sh, generator=g) * 1e-4 + 1e-6 for sh in shapes]
    agg_ref.fedopt_update(p2, d2, v2, msgs, opt, lr, betas, tau)
    exp_t = _flat(p2)
    theta0 = _flat([p.data for p in make_model(shapes, 1).parameters()])
    upd = np.abs(exp_t.astype(np.float64) - theta0)
    err = np.abs(exp_t.astype(np.float64) - got_theta.astype(np.float64))
    assert np.all(err <= 1e-6 * upd + np.spacing(np.abs(exp_t)))


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("opt,lr,betas,tau", OPTS)
@pytest.mark.parametrize("where", ["cuda:0", "host"])
def test_host_server_fedopt_update_matches_reference(tag, shapes, opt, lr, betas, tau, where):
    """FedOptServer.update (_fedopt.py:196-240) through FedOptUpdateMixin on a CPU server, 10 clients at config-1
    shapes: delta (and FedAvg's theta) bit-exact with agg.npz, the server's tensors still CPU tensors, updated in
    place (the same Parameter objects)."""
    msgs = make_msgs(shapes, 10, 3, "delta_parameters")
    s = _fedopt_server(shapes, opt, lr, betas, tau, _msgs_on(msgs, "delta_parameters", where))
    params = list(s.model.parameters())
    s.update()
    assert all(p.device.type == "cpu" for p in s.model.parameters())
    assert all(a is b for a, b in zip(params, s.model.parameters()))
    assert all(t.device.type == "cpu" for t in s.delta_parameters)
    assert _sha(s.delta_parameters) == str(AGG[f"fedopt_{opt}_{tag}|delta|sha"]), "delta average must be bit-exact"
    if opt == "avg":
        assert _sha(params) == str(AGG[f"fedopt_{opt}_{tag}|theta|sha"]), "FedAvg must be bit-exact"
    else:
        _check_adaptive_theta(shapes, opt, lr, betas, tau, msgs, _flat(params))


def test_host_server_rounds_track_host_side_writes():
    """Several rounds on one adopted server: between rounds the reference's own CPU code writes the server tensors
    (``p.data.add_`` — which does not bump a version counter — and a ``.data`` reassignment as Node.set_parameters
    does, nodes.py:461); every round must see those writes and equal the CPU oracle run on the same sequence."""
    shapes = CONFIG1_SHAPES
    s = _fedopt_server(shapes, "adam", 0.01, (0.9, 0.99), 1e-3, [])
    p2 = [p.data.clone() for p in s.model.parameters()]
    d2 = [t.clone() for t in s.delta_parameters]
    v2 = [t.clone() for t in s.v_parameters]
    for r in range(4):
        msgs = make_msgs(shapes, 7, 100 + r, "delta_parameters")
        s._received_messages = _msgs_on(msgs, "delta_parameters", "cuda:0")
        s.update()
        agg_ref.fedopt_update(p2, d2, v2, msgs, "adam", 0.01, (0.9, 0.99), 1e-3)
        # delta and v are bit-exact folds / steps; theta within the adaptive tolerance, then re-synchronised so the
        # rounds stay comparable
        assert np.array_equal(_flat(s.delta_parameters).view(np.int32), _flat(d2).view(np.int32))
        got = _flat(s.model.parameters())
        exp = _flat(p2)
        assert np.allclose(got, exp, rtol=1e-5, atol=1e-7)
        with torch.no_grad():
            for p, q in zip(s.model.parameters(), p2):
                p.data.copy_(q)
        # host-side writes between rounds
        if r == 1:
            for p in s.model.parameters():
                p.data.add_(0.5)
            for q in p2:
                q.add_(0.5)
        if r == 2:
            first = next(iter(s.model.parameters()))
            first.data = first.data.detach().clone() * 2  # reassigned storage (Node.set_parameters)
            p2[0] = p2[0] * 2


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("size_aware", [False, True])
@pytest.mark.parametrize("inertia", [0.0, 0.3])
@pytest.mark.parametrize("where", ["cuda:0", "host"])
def test_host_server_avg_parameters_matches_reference(tag, shapes, size_aware, inertia, where):
    s = _server_cls()()
    s.model = make_model(shapes, 4)
    s._received_messages = _msgs_on(make_msgs(shapes, 10, 5, "parameters"), "parameters", where)
    s.avg_parameters(size_aware=size_aware, inertia=inertia)
    assert all(p.device.type == "cpu" for p in s.model.parameters())
    assert _sha(list(s.model.parameters())) == str(AGG[f"avgp_{int(size_aware)}_{inertia}_{tag}|theta|sha"])


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("where", ["cuda:0", "host"])
def test_host_server_update_gradients_matches_reference(tag, shapes, where):
    s = _server_cls()()
    s.model = make_model(shapes, 6)
    s._received_messages = _msgs_on(make_msgs(shapes, 10, 7, "gradients"), "gradients", where)
    s.update_gradients()
    grads = [p.grad for p in s.model.parameters()]
    assert all(g.device.type == "cpu" for g in grads), "a CPU model gets CPU gradients (nodes.py:1172)"
    assert _sha(grads) == str(AGG[f"gradients_{tag}|grad|sha"])


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_host_server_add_parameters_functional_packed(tag, shapes):
    """The functional form on temporary ``p.data`` objects (not adoptable): staged by packing, written back into the
    parameters' own storage."""
    from fl_sim_amd import aggregation

    model = make_model(shapes, 4)
    msgs = make_msgs(shapes, 3, 9, "parameters")
    exp = [p.data.clone() for p in model.parameters()]
    for m in msgs:
        agg_ref.add_parameters(exp, m["parameters"], 0.25)
    for m in msgs:
        aggregation.add_parameters([p.data for p in model.parameters()], [t.cuda() for t in m["parameters"]], 0.25)
    assert np.array_equal(_flat(model.parameters()).view(np.int32), _flat(exp).view(np.int32))


@pytest.mark.parametrize("n_msgs", [17, 40])
def test_host_server_more_than_16_messages(n_msgs):
    """More messages than one flc_model_fold launch takes: chained launches, the step fused into the last one —
    the same chain as the CPU oracle (FedAvg, bit-exact)."""
    shapes = CONFIG1_SHAPES
    msgs = make_msgs(shapes, n_msgs, 11, "delta_parameters")
    s = _fedopt_server(shapes, "avg", 1, (0, 1), 1, _msgs_on(msgs, "delta_parameters", "cuda:0"))
    p2 = [p.data.clone() for p in s.model.parameters()]
    d2 = [t.clone() for t in s.delta_parameters]
    s.update()
    agg_ref.fedopt_update(p2, d2, None, msgs, "avg", 1, (0, 1), 1)
    assert np.array_equal(_flat(s.delta_parameters).view(np.int32), _flat(d2).view(np.int32))
    assert np.array_equal(_flat(s.model.parameters()).view(np.int32), _flat(p2).view(np.int32))


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_host_server_scaffold_matches_reference(tag, shapes):
    from fl_sim_amd.aggregation import SCAFFOLDUpdateMixin

    class Server(SCAFFOLDUpdateMixin):
        pass

    params, cvs, msgs = scaffold_inputs(shapes)
    s = Server()
    s.model = torch.nn.Module()
    for i, p in enumerate(params):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(p.clone()))
    s._control_variates = [c.clone() for c in cvs]
    s._received_messages = [{**m, "parameters_delta": [t.cuda() for t in m["parameters_delta"]]} for m in msgs]
    s._clients = list(range(SCAFFOLD_CFG["num_clients"]))
    s.config = _Cfg(lr=SCAFFOLD_CFG["lr"])
    s.update()
    assert _sha(list(s.model.parameters())) == str(AGGV[f"scaffold_{tag}|theta|sha"])
    assert _sha(s._control_variates) == str(AGGV[f"scaffold_{tag}|cv|sha"])
    assert all(c.device.type == "cpu" for c in s._control_variates)


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
def test_host_server_ifca_matches_reference(tag, shapes):
    from fl_sim_amd import aggregation

    centers, msgs = ifca_inputs(shapes)
    aggregation.ifca_update(centers, [{**m, "delta_parameters": [t.cuda() for t in m["delta_parameters"]]}
                                      for m in msgs], 4)
    for c in range(4):
        assert all(t.device.type == "cpu" for t in centers[c]["center_model_params"])
        assert _sha(centers[c]["center_model_params"]) == str(AGGV[f"ifca_{tag}|center{c}|sha"]), f"center {c}"
        assert centers[c]["client_ids"] == AGGV[f"ifca_{tag}|ids{c}"].tolist()


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("reg", ["l1_norm", "l2_norm_squared", "none"])
def test_host_server_feddr_matches_reference(tag, shapes, reg):
    from fl_sim_amd.aggregation import FedDRUpdateMixin

    class Server(FedDRUpdateMixin):
        pass

    params, ys, xts, msgs = feddr_inputs(shapes)
    s = Server()
    s.model = torch.nn.Module()
    for i, p in enumerate(params):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(p.clone()))
    s._y_parameters, s._x_til_parameters = [t.clone() for t in ys], [t.clone() for t in xts]
    s._received_messages = msgs
    s.config = _Cfg(alpha=FEDDR_CFG["alpha"], eta=FEDDR_CFG["eta"], num_clients=FEDDR_CFG["num_clients"], reg_type=reg)
    s.update()
    assert _sha(s._x_til_parameters) == str(AGGV[f"feddr_{reg}_{tag}|xtil|sha"])
    assert _sha(s._y_parameters) == str(AGGV[f"feddr_{reg}_{tag}|y|sha"])
    assert _sha(list(s.model.parameters())) == str(AGGV[f"feddr_{reg}_{tag}|theta|sha"])


from tests.golden.gen_golden import FEDDYN_CFG, PFEDME_BETAS, feddyn_inputs, pfedme_inputs  # noqa: E402


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("nm", [10, 20])
@pytest.mark.parametrize("where", ["host", "cuda"])
def test_host_server_feddyn_matches_reference(tag, shapes, nm, where):
    """FedDynServer.update on the reference's CPU server (model and h in host memory), messages on the device or the
    host: the mixin's result equals the reference's bit for bit."""
    from fl_sim_amd.aggregation import AggregationMixin, FedDynUpdateMixin

    class Server(FedDynUpdateMixin, AggregationMixin):
        pass

    params, hs, msgs = feddyn_inputs(shapes, nm)
    s = Server()
    s.model = torch.nn.Module()
    for i, p in enumerate(params):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(p.clone()))
    s.h_params = [t.clone() for t in hs]
    s._received_messages = _msgs_on(msgs, "parameters", where)
    s.config = _Cfg(**FEDDYN_CFG)
    s.update()
    assert all(p.device.type == "cpu" for p in s.model.parameters()) and all(h.device.type == "cpu" for h in s.h_params)
    assert _sha(s.h_params) == str(AGGV[f"feddyn_{nm}_{tag}|h|sha"])
    assert _sha(list(s.model.parameters())) == str(AGGV[f"feddyn_{nm}_{tag}|theta|sha"])


@pytest.mark.parametrize("tag,shapes", [("small", SMALL_SHAPES), ("config1", CONFIG1_SHAPES)])
@pytest.mark.parametrize("nm", [10, 20, 0])
@pytest.mark.parametrize("beta", PFEDME_BETAS)
def test_host_server_pfedme_matches_reference(tag, shapes, nm, beta):
    from fl_sim_amd.aggregation import AggregationMixin, pFedMeUpdateMixin

    class Server(pFedMeUpdateMixin, AggregationMixin):
        pass

    params, msgs = pfedme_inputs(shapes, nm)
    s = Server()
    s.model = torch.nn.Module()
    for i, p in enumerate(params):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(p.clone()))
    s._received_messages = _msgs_on(msgs, "parameters", "cuda")
    s.config = _Cfg(beta=beta)
    s.update()
    assert all(p.device.type == "cpu" for p in s.model.parameters())
    assert _sha(list(s.model.parameters())) == str(AGGV[f"pfedme_{beta}_{nm}_{tag}|theta|sha"])


def test_host_server_pinned_parameters_behave_as_cpu_tensors():
    """Adoption moves the storage into pinned host memory: the model still runs on the CPU (forward, in-place ops,
    state_dict round trip) with unchanged values."""
    shapes = SMALL_SHAPES
    msgs = make_msgs(shapes, 2, 3, "delta_parameters")
    s = _fedopt_server(shapes, "avg", 1, (0, 1), 1, _msgs_on(msgs, "delta_parameters", "cuda:0"))
    before = _flat(s.model.parameters())
    from fl_sim_amd.aggregation import _adopt

    _adopt([list(s.model.parameters()), s.delta_parameters])
    assert np.array_equal(_flat(s.model.parameters()), before)
    assert all(p.is_pinned() for p in s.model.parameters())
    sd = {k: v.clone() for k, v in s.model.state_dict().items()}
    with torch.no_grad():
        for p in s.model.parameters():
            p.mul_(2)
    s.model.load_state_dict(sd)
    assert np.array_equal(_flat(s.model.parameters()), before)
    assert all(p.is_pinned() for p in s.model.parameters()), "load_state_dict copies in place"


def test_host_server_zero_copy_is_taken(staging_mode):
    """The adopted mirror of a host server works on the pinned buffer in place when zero-copy is on (the device alias
    shares the host tensors' memory), and keeps a separate device buffer when it is off."""
    from fl_sim_amd import hoststage

    params = [torch.randn(5, 7), torch.randn(3)]
    m = hoststage.adopt([params], torch.device("cuda", 0))
    assert m is not None and m.zero_copy == (staging_mode == "zero_copy"), hoststage.ZERO_COPY_ERROR
    if m.zero_copy:
        assert m.dev.is_cuda and m.dev.data_ptr() == m.host.data_ptr() == params[0].data_ptr()
        m.dev_views(0)[1].fill_(2.5)  # a device-side write lands in the host tensor itself
        torch.cuda.synchronize()
        assert torch.equal(params[1], torch.full((3,), 2.5))
