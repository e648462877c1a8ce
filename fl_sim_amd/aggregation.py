"""Server-side aggregation on MI355X: the reference's ``Server`` aggregation methods as fused kernels.

Functional forms (explicit parameter lists) and a mixin that drops into the reference's ``Server``
subclasses unchanged (``class MyServer(AggregationMixin, FedAvgServer)``):

* ``add_parameters``      — nodes.py:1116-1132   ``server_param.add_(param, alpha=ratio)``
* ``avg_parameters``      — nodes.py:1134-1163   ``θ *= inertia; θ += Σ_m ratio_m · p_m``
* ``update_gradients``    — nodes.py:1165-1180   ``grad = Σ_m (ts_m / Σts) · g_m``
* ``fedopt_update``       — _fedopt.py:196-265   ``δ = β0 δ + Σ_m (1-β0)/n · δ_m`` then the
                                                  avg / adagrad / yogi / adam server step

Each tensor is folded in ONE launch (``flc_weighted_sum``): one read per message, one write, the
fmaf chain in message order — bit-identical to the reference's sequential ``add_`` loop, which torch
evaluates as one fp32 fma per element per message.  Scalars are formed in Python double exactly as
the reference forms them and rounded to fp32 at the boundary, as torch does.
"""

from __future__ import annotations

from typing import Iterable, List, Mapping, Optional, Sequence

import torch

from . import codec


def _params(ps) -> List[torch.Tensor]:
    return [p.data if isinstance(p, torch.nn.Parameter) else p for p in ps]


def _on(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    t = t.detach()
    return t if t.device == device else t.to(device)


def add_parameters(server_params: Iterable[torch.Tensor], params: Iterable[torch.Tensor], ratio: float) -> None:
    """nodes.py:1116-1132."""
    for sp, p in zip(_params(server_params), params):
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
    grads = []
    for j, mp in enumerate(model_params):
        g0 = messages[0]["gradients"][j]
        dev = mp.device if mp.device.type == "cuda" else g0.device
        g = torch.empty(g0.shape, dtype=torch.float32, device=dev)
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
    for j, dp in enumerate(delta_parameters):
        srcs = [_on(m["delta_parameters"][j], dp.device) for m in messages]
        codec.weighted_sum(dp, srcs, [alpha] * len(srcs), init_mode=0, beta=betas[0])
    ps = _params(model_params)
    for j, (sp, dp) in enumerate(zip(ps, delta_parameters)):
        vp = None if (v_parameters is None or opt == "avg") else v_parameters[j]
        codec.fedopt_step(sp, dp, vp, opt if vp is not None else "avg", lr, betas[1], tau)


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
