"""ORACLE — test infrastructure only.  Never imported by the product package (fl_sim_amd/).

torch-CPU restatement of the reference's server aggregation, operation for operation:
``Server.add_parameters`` / ``avg_parameters`` / ``update_gradients`` (fl_sim/nodes.py:1116-1180)
and ``FedOptServer.update`` with its avg/adagrad/yogi/adam tails (fl_sim/algorithms/fedopt/
_fedopt.py:196-265).  It runs the same torch CPU kernels the reference runs (``mul_``, ``add_`` with
``alpha``, ``addcmul_``, ``addcdiv_``), so it rounds exactly where the reference rounds.  Pinned by
``tests/golden/agg_*.npz``, produced by executing the reference's own method bodies
(``tests/golden/gen_golden.py``).
"""

from __future__ import annotations

from typing import List, Mapping, Optional, Sequence

import torch


def add_parameters(params: Sequence[torch.Tensor], others: Sequence[torch.Tensor], ratio: float) -> None:
    for p, o in zip(params, others):  # nodes.py:1131-1132
        p.add_(o.detach().clone(), alpha=ratio)


def avg_parameters(params: Sequence[torch.Tensor], messages: Sequence[Mapping], size_aware=False, inertia=0.0,
                   key="parameters") -> None:
    assert 0.0 <= inertia < 1.0
    if len(messages) == 0:
        return
    for p in params:  # nodes.py:1158-1159
        p.mul_(inertia)
    total = sum(m["train_samples"] for m in messages)
    for m in messages:  # nodes.py:1161-1163
        ratio = (m["train_samples"] / total if size_aware else 1 / len(messages)) * (1 - inertia)
        add_parameters(params, m[key], ratio)


def update_gradients(shapes_like: Sequence[torch.Tensor], messages: Sequence[Mapping]) -> Optional[List[torch.Tensor]]:
    if len(messages) == 0:
        return None
    grads = [torch.zeros_like(g) for g in messages[0]["gradients"]]  # nodes.py:1173-1174
    total = sum(m["train_samples"] for m in messages)
    for m in messages:  # nodes.py:1176-1180
        for g, gd in zip(grads, m["gradients"]):
            g.add_(gd.detach().clone(), alpha=m["train_samples"] / total)
    return grads


def fedopt_update(params, delta_params, v_params, messages, optimizer: str, lr: float, betas, tau: float) -> None:
    for idx, dp in enumerate(delta_params):  # _fedopt.py:202-208
        dp.mul_(betas[0])
        for m in messages:
            dp.add_(m["delta_parameters"][idx].detach().clone(), alpha=(1 - betas[0]) / len(messages))
    opt = optimizer.lower()
    if opt == "adagrad":  # _fedopt.py:248-250
        for vp, dp in zip(v_params, delta_params):
            vp.add_(dp.pow(2))
    elif opt == "yogi":  # _fedopt.py:252-258
        for vp, dp in zip(v_params, delta_params):
            vp.addcmul_(dp.pow(2), (vp - dp.pow(2)).sign(), value=-(1 - betas[1]))
    elif opt == "adam":  # _fedopt.py:260-263
        for vp, dp in zip(v_params, delta_params):
            vp.mul_(betas[1]).add_(dp.pow(2), alpha=1 - betas[1])
    if opt == "avg" or v_params is None:  # _fedopt.py:231-233
        for sp, dp in zip(params, delta_params):
            sp.add_(dp, alpha=lr)
    else:  # _fedopt.py:234-239
        for sp, dp, vp in zip(params, delta_params, v_params):
            sp.addcdiv_(dp, vp.sqrt() + tau, value=lr)
