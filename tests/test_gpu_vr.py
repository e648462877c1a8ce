"""GPU parity of the variance-reduced servers' update in one launch (flc_avg_and_gradients,
aggregation.avg_parameters_and_gradients and the VRUpdateMixin family): FedProx / FedPD / ProxSkip / pFedMac
``update`` against the reference's own (tests/golden/agg_vr.npz, gen_golden.py ``gen_vr``), bit for bit, with and
without ``vr``, 10 and 20 messages (chained launches), on a device- and a host-resident model."""

import types

import numpy as np
import pytest
import torch

from tests import golden_cases as gc
from tests.golden.gen_golden import CONFIG1_SHAPES, PFEDMAC_BETA, SMALL_SHAPES, VR_SERVERS, vr_inputs

pytestmark = pytest.mark.gpu
VR = np.load(f"{gc.GOLDEN}/agg_vr.npz", allow_pickle=False)


def _same(key, ts):
    a = torch.cat([t.detach().reshape(-1).cpu() for t in ts]).numpy()
    if key + "|out" in VR.files:
        return gc.same_bits(a, VR[key + "|out"])
    return gc.sha(a) == str(VR[key + "|sha"])


def _mixin(name):
    from fl_sim_amd import aggregation as agg

    return {"fedprox": agg.FedProxUpdateMixin, "fedpd": agg.FedPDUpdateMixin, "proxskip": agg.ProxSkipUpdateMixin,
            "pfedmac": agg.pFedMacUpdateMixin}[name]


@pytest.mark.parametrize("where", ["device", "host"])
@pytest.mark.parametrize("tag", ["small", "config1"])
@pytest.mark.parametrize("nm", [10, 20])
@pytest.mark.parametrize("vr", [True, False])
@pytest.mark.parametrize("name", list(VR_SERVERS))
def test_vr_server_update_matches_reference(name, vr, nm, tag, where):
    shapes = SMALL_SHAPES if tag == "small" else CONFIG1_SHAPES
    params, msgs = vr_inputs(shapes, nm)

    class Server(_mixin(name)):
        pass

    s = Server()
    dev = "cuda" if where == "device" else "cpu"
    s.model = torch.nn.Module()
    for i, t in enumerate(params):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(t.clone().to(dev)))
    s.config = types.SimpleNamespace(vr=vr, beta=PFEDMAC_BETA)
    s._received_messages = [dict(m, parameters=[t.cuda() for t in m["parameters"]],
                                 gradients=[t.cuda() for t in m["gradients"]]) for m in msgs]
    s.update()
    key = f"vr_{name}_{int(vr)}_{nm}_{tag}"
    assert _same(key + "|theta", list(s.model.parameters()))
    if vr:
        assert _same(key + "|grad", [p.grad for p in s.model.parameters()])
        assert all(p.grad.device.type == dev for p in s.model.parameters())
    if name == "fedpd":
        assert s._communicated_clients == [m["client_id"] for m in msgs]


@pytest.mark.parametrize("size_aware,inertia", [(False, 0.0), (True, 0.3)])
def test_avg_parameters_and_gradients_equals_the_two_calls(size_aware, inertia):
    """The fused launch against avg_parameters then update_gradients, including misaligned (non-16-B) tensors and
    a message held on the host (moved), bit for bit."""
    from fl_sim_amd import aggregation as agg

    g = torch.Generator().manual_seed(5)
    sizes = [3, 1027, 5, 4096, 7, 1]
    base = torch.randn(sum(sizes) + 1, generator=g).cuda()
    ps, off = [], 1
    for n in sizes:
        ps.append(base[off:off + n])
        off += n
    msgs = [{"parameters": [torch.randn(n, generator=g).cuda() for n in sizes],
             "gradients": [torch.randn(n, generator=g).cuda() for n in sizes], "train_samples": 10 * (i + 3)}
            for i in range(18)]
    msgs[4]["parameters"][2] = msgs[4]["parameters"][2].cpu()
    a = [p.clone() for p in ps]
    ga = agg.avg_parameters_and_gradients(a, msgs, size_aware, inertia)
    b = [p.clone() for p in ps]
    agg.avg_parameters(b, msgs, size_aware, inertia)
    gb = agg.update_gradients(b, msgs)
    for x, y in zip(a + ga, b + gb):
        assert gc.same_bits(x.cpu().numpy(), y.cpu().numpy())


@pytest.mark.parametrize("kind", ["parameter", "tensor"])
def test_avg_parameters_and_gradients_one_call_sets_grad(kind):
    """Everything on the device: the one C call (the fold, the gradients' flat buffer and per-parameter views, every
    `.grad` set in C++) against avg_parameters then update_gradients, on nn.Parameters and on plain tensors."""
    from fl_sim_amd import aggregation as agg

    g = torch.Generator().manual_seed(6)
    shapes = [(16, 1, 5, 5), (16,), (256, 37), (10,)]
    th = [torch.randn(s, generator=g).cuda() for s in shapes]
    msgs = [{"parameters": [t + torch.randn(t.shape, generator=g).cuda() * 1e-2 for t in th],
             "gradients": [torch.randn(t.shape, generator=g).cuda() for t in th], "train_samples": 7 * (i + 2)}
            for i in range(12)]
    make = (lambda t: torch.nn.Parameter(t.clone())) if kind == "parameter" else (lambda t: t.clone())
    a, b = [make(t) for t in th], [make(t) for t in th]
    ga = agg.avg_parameters_and_gradients(a, msgs, True, 0.2)
    agg.avg_parameters(b, msgs, True, 0.2)
    gb = agg.update_gradients(b, msgs)
    for j, (x, y) in enumerate(zip(a, b)):
        assert gc.same_bits(x.detach().cpu().numpy(), y.detach().cpu().numpy()), j
        assert x.grad is not None and x.grad.shape == shapes[j] and x.grad.data_ptr() == ga[j].data_ptr()
        assert gc.same_bits(x.grad.cpu().numpy(), y.grad.cpu().numpy()) and gc.same_bits(ga[j].cpu().numpy(),
                                                                                           gb[j].cpu().numpy())
