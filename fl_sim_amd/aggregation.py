"""Server-side aggregation on MI355X: the reference's ``Server`` aggregation methods as fused kernels.

Functional forms (explicit parameter lists) and a mixin that drops into the reference's ``Server``
subclasses unchanged (``class MyServer(AggregationMixin, FedAvgServer)``):

* ``add_parameters``      — nodes.py:1116-1132   ``server_param.add_(param, alpha=ratio)``
* ``avg_parameters``      — nodes.py:1134-1163   ``θ *= inertia; θ += Σ_m ratio_m · p_m``
* ``update_gradients``    — nodes.py:1165-1180   ``grad = Σ_m (ts_m / Σts) · g_m``
* ``fedopt_update``       — _fedopt.py:196-265   ``δ = β0 δ + Σ_m (1-β0)/n · δ_m`` then the
                                                  avg / adagrad / yogi / adam server step
* ``scaffold_update``     — _scaffold.py:158-167 ``θ += Σ_m lr/n · Δθ_m``, ``c += Σ_m 1/N · Δc_m``
* ``ifca_update``         — _ifca.py:167-195     per cluster ``center += Σ_{m in cluster} 1/size · δ_m``
                                                  (and the reference's client-id bookkeeping)
* ``feddr_update``        — _feddr.py:166-190    ``y`` relaxation, ``x̃`` fold, ``θ = prox(c_x x̃ + c_y y)``

A whole model is folded in ONE launch (``flc_model_fold``, up to 16 messages; FedOpt's optimizer step fused into
the same pass), else each tensor in one launch (``flc_weighted_sum``): one read per message, one write, the fmaf chain
in message order — bit-identical to the reference's sequential ``add_`` loop, which torch evaluates as one fp32 fma
per element per message.  Scalars are formed in Python double exactly as the reference forms them and rounded to fp32
at the boundary, as torch does.
"""

from __future__ import annotations

import math
from typing import Iterable, List, Mapping, Optional, Sequence

import torch

from . import _lib, codec


def _params(ps) -> List[torch.Tensor]:
    return [p.data if isinstance(p, torch.nn.Parameter) else p for p in ps]


def _on(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    t = t.detach()
    return t if t.device == device else t.to(device)


def _model_device(tensors: Sequence[torch.Tensor]) -> Optional[int]:
    """The index of the one HIP device all of a model's tensors live on (contiguous fp32), or None (then per-tensor
    launches)."""
    dev = None
    for t in tensors:
        if not (t.is_cuda and t.dtype is torch.float32 and t.is_contiguous()):
            return None
        d = t.get_device()
        if dev is None:
            dev = d
        elif d != dev:
            return None
    return dev


def _fold(dsts: Sequence[torch.Tensor], msg_tensors: Sequence[Sequence[torch.Tensor]], weights: Sequence[float],
          init_mode: int, beta: float = 0.0, **step) -> bool:
    """The whole model in one flc_model_fold launch when it qualifies (one device, <= 16 messages); False otherwise."""
    dev = _model_device(list(dsts) + list(step.get("theta") or []) + list(step.get("v") or []))
    if dev is None or not dsts or len(msg_tensors) > codec.MODEL_FOLD_MAX_SRC:
        return False
    if codec._model_fold_op() is not None:
        # the op checks every tensor in C++ before launching anything: with the messages already on the model's
        # device (the usual case) that is the whole host cost; otherwise it raises TypeError and they are moved below
        try:
            codec.model_fold(dsts, msg_tensors, weights, init_mode, beta, **step)
            return True
        except TypeError:
            pass
    srcs = [[t if (t.is_cuda and t.get_device() == dev) else t.detach().to(f"cuda:{dev}") for t in mt]
            for mt in msg_tensors]
    codec.model_fold(dsts, srcs, weights, init_mode, beta, **step)
    return True


def add_parameters(server_params: Iterable[torch.Tensor], params: Iterable[torch.Tensor], ratio: float) -> None:
    """nodes.py:1116-1132."""
    sps, ps = _params(server_params), list(params)
    if _fold(sps, [ps], [ratio], 2):
        return
    for sp, p in zip(sps, ps):
        codec.weighted_sum(sp, [_on(p, sp.device)], [ratio], init_mode=2)


def avg_parameters(server_params: Sequence[torch.Tensor], messages: Sequence[Mapping], size_aware: bool = False,
                   inertia: float = 0.0, key: str = "parameters") -> None:
    """nodes.py:1134-1163 (weights formed in double, message order preserved)."""
    assert 0.0 <= inertia < 1.0, "`inertia` should be in [0, 1)"
    if len(messages) == 0:
        return
    total_samples = sum([m["train_samples"] for m in messages])
    ratios = [
        (m["train_samples"] / total_samples if size_aware else 1 / len(messages)) * (1 - inertia) for m in messages
    ]
    if _fold(_params(server_params), [m[key] for m in messages], ratios, 0, inertia):
        return
    for j, sp in enumerate(_params(server_params)):
        srcs = [_on(m[key][j], sp.device) for m in messages]
        codec.weighted_sum(sp, srcs, ratios, init_mode=0, beta=inertia)


def update_gradients(model_params: Sequence[torch.Tensor], messages: Sequence[Mapping]) -> Optional[List[torch.Tensor]]:
    """nodes.py:1165-1180: sets ``.grad`` of each model parameter to the sample-weighted gradient sum."""
    if len(messages) == 0:
        return None
    assert all(["gradients" in m for m in messages]), "some clients have not sent gradients yet"
    total_samples = sum([m["train_samples"] for m in messages])
    weights = [m["train_samples"] / total_samples for m in messages]
    g0s = messages[0]["gradients"]
    devs = {mp.device if mp.device.type == "cuda" else g.device for mp, g in zip(model_params, g0s)}
    if len(devs) == 1 and next(iter(devs)).type == "cuda":
        dev = next(iter(devs))
        gs = [torch.empty(g.shape, dtype=g.dtype, device=dev) for g in g0s]
        if _fold(gs, [m["gradients"] for m in messages], weights, 1):
            for mp, g in zip(model_params, gs):
                if isinstance(mp, torch.Tensor) and mp.requires_grad:
                    mp.grad = g
            return gs
    grads = []
    for j, mp in enumerate(model_params):
        g0 = messages[0]["gradients"][j]
        dev = mp.device if mp.device.type == "cuda" else g0.device
        g = torch.empty(g0.shape, dtype=g0.dtype, device=dev)
        codec.weighted_sum(g, [_on(m["gradients"][j], dev) for m in messages], weights, init_mode=1)
        if isinstance(mp, torch.Tensor) and mp.requires_grad:
            mp.grad = g
        grads.append(g)
    return grads


def fedopt_update(model_params: Sequence[torch.Tensor], delta_parameters: Sequence[torch.Tensor],
                  v_parameters: Optional[Sequence[torch.Tensor]], messages: Sequence[Mapping], optimizer: str,
                  lr: float, betas: Sequence[float], tau: float) -> None:
    """_fedopt.py:196-265 (FedAvg: optimizer="avg", lr=1, betas=(0, 1))."""
    opt = optimizer.lower()
    if opt not in ("avg", "adagrad", "yogi", "adam"):
        raise ValueError(f"Unknown optimizer: {optimizer}")
    alpha = (1 - betas[0]) / len(messages) if len(messages) else 0.0
    ps = _params(model_params)
    vps = None if (v_parameters is None or opt == "avg") else list(v_parameters)
    if _fold(list(delta_parameters), [m["delta_parameters"] for m in messages], [alpha] * len(messages), 0, betas[0],
             theta=ps, v=vps, opt=opt if vps is not None else "avg", lr=lr, beta2=betas[1], tau=tau):
        return  # the delta average and the optimizer step of every tensor in one launch
    for j, dp in enumerate(delta_parameters):
        srcs = [_on(m["delta_parameters"][j], dp.device) for m in messages]
        codec.weighted_sum(dp, srcs, [alpha] * len(srcs), init_mode=0, beta=betas[0])
    ps = _params(model_params)
    for j, (sp, dp) in enumerate(zip(ps, delta_parameters)):
        vp = None if (v_parameters is None or opt == "avg") else v_parameters[j]
        codec.fedopt_step(sp, dp, vp, opt if vp is not None else "avg", lr, betas[1], tau)


def scaffold_update(model_params: Sequence[torch.Tensor], control_variates: Sequence[torch.Tensor],
                    messages: Sequence[Mapping], lr: float, num_clients: int) -> None:
    """_scaffold.py:158-167.  The reference interleaves the two folds per message; they touch different tensors,
    so each tensor's fmaf chain (message order) is the same when folded in one launch per tensor."""
    if len(messages) == 0:
        raise ZeroDivisionError("division by zero")  # ratio_p = lr / len(messages) in the reference
    ratio_p = lr / len(messages)
    ratio_c = 1 / num_clients
    ps, cvs = _params(model_params), list(control_variates)
    if _model_device(ps + cvs) is not None and ps and cvs and len(messages) <= codec.MODEL_FOLD_MAX_SRC:
        _fold(ps, [m["parameters_delta"] for m in messages], [ratio_p] * len(messages), 2)
        _fold(cvs, [m["control_variates_delta"] for m in messages], [ratio_c] * len(messages), 2)
        return
    for j, sp in enumerate(_params(model_params)):
        codec.weighted_sum(sp, [_on(m["parameters_delta"][j], sp.device) for m in messages], [ratio_p] * len(messages),
                           init_mode=2)
    for j, cv in enumerate(control_variates):
        codec.weighted_sum(cv, [_on(m["control_variates_delta"][j], cv.device) for m in messages],
                           [ratio_c] * len(messages), init_mode=2)


def ifca_update(cluster_centers: Mapping[int, dict], messages: Sequence[Mapping], num_clusters: int) -> None:
    """_ifca.py:167-195 on ``{cluster_id: {"center_model_params": [...], "client_ids": [...]}}``, in place.

    Host bookkeeping as in the reference: the round's members are listed, idle members of the previous round rejoin
    their cluster, and each member is appended once more while its delta is folded (the reference's duplicate
    entries are kept, so downstream code sees the same lists).  Each center tensor is folded in one launch."""
    prev = {c: list(v["client_ids"]) for c, v in cluster_centers.items()}
    for v in cluster_centers.values():
        v["client_ids"] = []
    sizes = {c: 0 for c in range(num_clusters)}
    members: dict = {}
    for m in messages:
        sizes[m["cluster_id"]] += 1
        cluster_centers[m["cluster_id"]]["client_ids"].append(m["client_id"])
        members.setdefault(m["cluster_id"], []).append(m)
    collected = set(i for v in cluster_centers.values() for i in v["client_ids"])
    for c, v in cluster_centers.items():
        v["client_ids"].extend(i for i in prev[c] if i not in collected)
    for c, ms in members.items():
        for j, p in enumerate(_params(cluster_centers[c]["center_model_params"])):
            codec.weighted_sum(p, [_on(m["delta_parameters"][j], p.device) for m in ms], [1 / sizes[c]] * len(ms),
                               init_mode=2)
    for m in messages:
        cluster_centers[m["cluster_id"]]["client_ids"].append(m["client_id"])


_PROX_KIND = {"l1": "l1", "l2": "l2", "l2squared": "l2squared", "no": "none", "empty": "none", "zero": "none",
              "none": "none", "null": "none"}
_LINF = ("linf", "inf", "linfinity", "infinity", "linfty", "infty")


def feddr_update(model_params: Sequence[torch.Tensor], y_params: Sequence[torch.Tensor],
                 x_til_params: Sequence[torch.Tensor], messages: Sequence[Mapping], alpha: float, eta: float,
                 num_clients: int, reg_type: str) -> None:
    """_feddr.py:166-190 with the regularizer get_regularizer(reg_type, eta·N/(N+1)) builds (_feddr.py:147-150).

    Per tensor: the x̃ fold (flc_weighted_sum), then one pass for the y relaxation, the combination and the
    proximal step (flc_feddr_combine).  L1 and L2-squared proxes are fused; L2's factor needs the norm of the
    combined θ over all tensors (an fp64 sum of squares per tensor; the reference sums fp32 per-tensor sums, so
    this one is equal to within rounding, not bit for bit), then θ is scaled in a second pass."""
    import re

    kind = re.sub("regularizer|norm|[\\s\\_\\-]+", "", reg_type.lower())
    if kind in _LINF:
        raise NotImplementedError("L-infinity norm is not implemented yet")
    if kind not in _PROX_KIND:
        raise ValueError(f"Unknown regularizer type: {reg_type}")
    kind = _PROX_KIND[kind]
    coeff = eta * num_clients / (num_clients + 1)
    total = sum([m["train_samples"] for m in messages])
    weights = [m["train_samples"] / total for m in messages]
    for j, xt in enumerate(x_til_params):
        codec.weighted_sum(xt, [_on(m["x_hat_delta"][j], xt.device) for m in messages], weights, init_mode=2)
    cx, cy = coeff / eta, 1 / (num_clients + 1)
    if kind == "l1":
        prox, pc = _lib.FLC_PROX_L1, coeff
    elif kind == "l2squared":
        prox, pc = _lib.FLC_PROX_SCALE, 1 / (1 + 2 * coeff)
    else:
        prox, pc = _lib.FLC_PROX_NONE, 0.0
    ps = _params(model_params)
    for sp, yp, xt in zip(ps, y_params, x_til_params):
        codec.feddr_combine(sp, yp, xt, alpha, cx, cy, prox, pc)
    if kind == "l2":
        sq = 0.0
        for sp in ps:
            nrm = codec.quant_norm_f64(sp, 2) if sp.dtype == torch.float64 else codec.quant_norm(sp.reshape(1, -1), 2)
            sq += float(nrm.item()) ** 2
        norm = coeff * math.sqrt(sq)
        f = max(0, 1 - coeff / norm)
        for sp in ps:
            codec.weighted_sum(sp, [], [], init_mode=0, beta=f)


class AggregationMixin:
    """Mix in before a reference ``Server`` subclass to run its aggregation on the device.

    Requires the server model on a HIP device (``self.model`` parameters on ``cuda:k``).
    """

    def add_parameters(self, params, ratio: float) -> None:  # nodes.py:1116
        add_parameters(self.model.parameters(), params, ratio)

    def avg_parameters(self, size_aware: bool = False, inertia: float = 0.0) -> None:  # nodes.py:1134
        avg_parameters(list(self.model.parameters()), self._received_messages, size_aware, inertia)

    def update_gradients(self) -> None:  # nodes.py:1165
        update_gradients(list(self.model.parameters()), self._received_messages)


class FedOptUpdateMixin:
    """Device ``update()`` for the reference's ``FedOptServer`` family (_fedopt.py:196-240)."""

    def update(self) -> None:
        fedopt_update(list(self.model.parameters()), self.delta_parameters, self.v_parameters,
                      self._received_messages, self.config.optimizer, self.config.lr, self.config.betas,
                      self.config.tau)


class SCAFFOLDUpdateMixin:
    """Device ``update()`` for the reference's ``SCAFFOLDServer`` (_scaffold.py:158-167)."""

    def update(self) -> None:
        scaffold_update(list(self.model.parameters()), self._control_variates, self._received_messages,
                        self.config.lr, len(self._clients))


class IFCAUpdateMixin:
    """Device ``update()`` for the reference's ``IFCAServer`` (_ifca.py:167-195)."""

    def update(self) -> None:
        ifca_update(self._cluster_centers, self._received_messages, self.config.num_clusters)


class FedDRUpdateMixin:
    """Device ``update()`` for the reference's ``FedDRServer`` (_feddr.py:166-190)."""

    def update(self) -> None:
        feddr_update(list(self.model.parameters()), self._y_parameters, self._x_til_parameters,
                     self._received_messages, self.config.alpha, self.config.eta, self.config.num_clients,
                     self.config.reg_type)
