"""ORACLE — test infrastructure only.  Never imported by the product package (fl_sim_amd/).

torch-CPU restatement of the reference's server aggregation, operation for operation:
``Server.add_parameters`` / ``avg_parameters`` / ``update_gradients`` (fl_sim/nodes.py:1116-1180)
and ``FedOptServer.update`` with its avg/adagrad/yogi/adam tails (fl_sim/algorithms/fedopt/
_fedopt.py:196-265); the f4 variants ``SCAFFOLDServer.update`` (scaffold/_scaffold.py:158-167), ``IFCAServer.update``
(ifca/_ifca.py:167-195) and ``FedDRServer.update`` (feddr/_feddr.py:166-190) with the regularizers' proximal steps
(regularizers/regularizers.py:146-200); and (round 5) ``FedDynServer.update`` (feddyn/_feddyn.py:172-184) and
``pFedMeServer.update`` (pfedme/_pfedme.py:166-175).  It runs the same torch CPU kernels the reference runs (``mul_``, ``add_`` with
``alpha``, ``addcmul_``, ``addcdiv_``), so it rounds exactly where the reference rounds.  Pinned by
``tests/golden/agg.npz`` and ``agg_variants.npz``, produced by executing the reference's own method bodies
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


# ------------------------------------------------------------------------------------------ f4 variants
def scaffold_update(params, control_variates, messages, lr: float, num_clients: int) -> None:
    ratio_p = lr / len(messages)  # _scaffold.py:160-161
    ratio_c = 1 / num_clients
    for m in messages:  # _scaffold.py:162-167: message order, parameters then control variates
        add_parameters(params, m["parameters_delta"], ratio_p)
        for cv, d in zip(control_variates, m["control_variates_delta"]):
            cv.add_(d.detach().clone(), alpha=ratio_c)


def ifca_update(centers: dict, messages, num_clusters: int) -> None:
    """``centers[c] = {"center_model_params": [...], "client_ids": [...]}``, updated in place."""
    prev = {c: list(v["client_ids"]) for c, v in centers.items()}  # _ifca.py:170
    for v in centers.values():
        v["client_ids"] = []
    sizes = {c: 0 for c in range(num_clusters)}
    for m in messages:  # _ifca.py:176-178
        sizes[m["cluster_id"]] += 1
        centers[m["cluster_id"]]["client_ids"].append(m["client_id"])
    collected = [i for v in centers.values() for i in v["client_ids"]]
    for c, v in centers.items():  # _ifca.py:182-185: idle members rejoin their cluster
        for i in prev[c]:
            if i not in collected:
                v["client_ids"].append(i)
    for m in messages:  # _ifca.py:187-195 (the client id is appended a second time, as in the reference)
        c = m["cluster_id"]
        for p, d in zip(centers[c]["center_model_params"], m["delta_parameters"]):
            p.add_(d.detach().clone(), alpha=1 / sizes[c])
        centers[c]["client_ids"].append(m["client_id"])


def prox(params, reg_type: str, coeff: float):
    """regularizers.py:146-200 (name normalisation of get_regularizer, regularizers.py:108)."""
    import math
    import re

    kind = re.sub("regularizer|norm|[\\s\\_\\-]+", "", reg_type.lower())
    if kind == "l1":
        return [p.sign() * (p.abs() - coeff).clamp(min=0) for p in params]
    if kind == "l2":
        norm = coeff * math.sqrt(sum([p.pow(2).sum().item() for p in params]))
        f = max(0, 1 - coeff / norm)
        return [f * p for p in params]
    if kind == "l2squared":
        return [(1 / (1 + 2 * coeff)) * p for p in params]
    if kind in ("no", "empty", "zero", "none", "null"):
        return list(params)
    if kind in ("linf", "inf", "linfinity", "infinity", "linfty", "infty"):
        raise NotImplementedError("L-infinity norm is not implemented yet")
    raise ValueError(f"Unknown regularizer type: {reg_type}")


def feddr_update(params, y_params, x_til_params, messages, alpha: float, eta: float, num_clients: int,
                 reg_type: str) -> None:
    coeff = eta * num_clients / (num_clients + 1)  # _feddr.py:147-150
    for yp, mp in zip(y_params, params):  # _feddr.py:169-170
        yp.add_(mp - yp, alpha=alpha)
    total = sum(m["train_samples"] for m in messages)
    for m in messages:  # _feddr.py:174-180
        for i, xt in enumerate(x_til_params):
            xt.add_(m["x_hat_delta"][i], alpha=m["train_samples"] / total)
    for mp, yp, xt in zip(params, y_params, x_til_params):  # _feddr.py:184-185
        mp.copy_((coeff / eta) * xt + (1 / (num_clients + 1)) * yp)
    for mp, p in zip(params, prox(params, reg_type, coeff)):  # _feddr.py:186-190
        mp.copy_(p)


def client_delta(local_params, cached_params):
    """FedOptClient.communicate (_fedopt.py:294-297): detached clones of the local parameters, minus the cached
    global ones via add_(alpha=-1)."""
    deltas = [p.detach().clone() for p in local_params]  # nodes.py:300-302
    for dp, rp in zip(deltas, cached_params):
        dp.add_(rp, alpha=-1)
    return deltas


def feddyn_update(params, h_params, messages, mu: float, num_clients: int) -> None:
    for m in messages:  # feddyn/_feddyn.py:174-180: h updated against the model before the average
        for hp, p, mp in zip(h_params, params, m["parameters"]):
            hp.add_(mp - p, alpha=-mu / num_clients)
    avg_parameters(params, messages)  # _feddyn.py:182
    # _feddyn.py:183-184: `p = p.add(...)` rebinds a local name; the model is not changed


def pfedme_update(params, messages, beta: float) -> None:
    previous = [p.detach().clone() for p in params]  # pfedme/_pfedme.py:166-167
    avg_parameters(params, messages)  # _pfedme.py:170
    for pre, p in zip(previous, params):  # _pfedme.py:173-174
        p.mul_(beta).add_(pre.detach().clone(), alpha=1 - beta)
