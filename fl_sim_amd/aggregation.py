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

A server whose model lives in host memory — the reference's own placement (nodes.py:606) — is served by the same
launches: its tensors are staged to the device and written back in place (``hoststage``; the mixins adopt the
server's tensors into one pinned buffer so that staging is one copy each way).

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

from . import _lib, codec, compressed, hoststage


def _params(ps) -> List[torch.Tensor]:
    return [p.data if isinstance(p, torch.nn.Parameter) else p for p in ps]


def _on(t: torch.Tensor, device: torch.device) -> torch.Tensor:
    t = t.detach()
    return t if t.device == device else t.to(device)


def _model_device(tensors: Sequence[torch.Tensor]) -> Optional[int]:
    """The HIP device index of a model whose first tensor is a contiguous fp32 HIP tensor, else None (then per-tensor
    launches).  Only the first tensor is looked at here: the model-fold op checks every tensor (device, dtype,
    contiguity, size) in C++ before it launches anything, and a model that fails those checks falls back to the
    per-tensor path in ``_fold`` — a model update is ~10-100 tensors, and a Python check per tensor cost more than the
    kernel."""
    if not tensors:
        return None
    t = tensors[0]
    if not (t.is_cuda and t.dtype is torch.float32):
        return None
    return t.get_device()


def _fold(dsts: Sequence[torch.Tensor], msg_tensors: Sequence, weights: Sequence[float], init_mode: int,
          beta: float = 0.0, key: Optional[str] = None, **step) -> bool:
    """The whole model in flc_model_fold launches when it qualifies (one device): one launch per 16 messages, the
    chain continued from the stored partial sums (init mode 2) and the FedOpt step fused into the last launch only —
    the same fmaf chain as one launch.  ``msg_tensors``: one tensor list per message, or (``key``) the messages
    themselves, each holding its list under ``key``.  False when the model does not qualify."""
    dev = _model_device(dsts)
    if dev is None:
        return False
    pf = codec._pyfold()
    if pf is not None:
        try:  # the common case in one C call: messages already on the model's device
            pf(dsts, msg_tensors, key, weights, init_mode, beta, step.get("theta"), step.get("v"),
               _lib.FLC_OPT[step.get("opt", "avg")], float(step.get("lr", 1.0)), float(step.get("beta2", 0.0)),
               float(step.get("tau", 0.0)))
            return True
        except TypeError:
            pass  # messages elsewhere (moved below) or a model the fold does not take (per-tensor launches)
    if key is not None:
        msg_tensors = [m[key] for m in msg_tensors]
    cap = codec.MODEL_FOLD_MAX_SRC
    launched = False  # a launch has written the model: from then on a failure has no clean fallback
    try:
        if len(msg_tensors) > cap:
            for c0 in range(0, len(msg_tensors) - cap, cap):
                _fold_one(dev, dsts, msg_tensors[c0:c0 + cap], weights[c0:c0 + cap], init_mode if c0 == 0 else 2,
                          beta)
                launched = True
                init_mode = 2  # (the chain continues from the stored partial sums)
            last = (len(msg_tensors) - 1) // cap * cap
            _fold_one(dev, dsts, msg_tensors[last:], weights[last:], 2, beta, **step)
            return True
        _fold_one(dev, dsts, msg_tensors, weights, init_mode, beta, **step)
    except TypeError:
        if launched:
            raise  # (a later chunk's tensors failed after an earlier launch ran)
        return False  # a model tensor the fold does not take (dtype, device, layout): per-tensor launches
    return True


def _fold_one(dev: int, dsts, msg_tensors, weights, init_mode: int, beta: float, **step) -> None:
    if codec._model_fold_op() is not None:
        # the op checks every tensor in C++ before launching anything: with the messages already on the model's
        # device (the usual case) that is the whole host cost; otherwise it raises TypeError and they are moved below
        try:
            codec.model_fold(dsts, msg_tensors, weights, init_mode, beta, **step)
            return
        except TypeError:
            pass
    srcs = [[t if (t.is_cuda and t.get_device() == dev) else t.detach().to(f"cuda:{dev}") for t in mt]
            for mt in msg_tensors]
    codec.model_fold(dsts, srcs, weights, init_mode, beta, **step)


def add_parameters(server_params: Iterable[torch.Tensor], params: Iterable[torch.Tensor], ratio: float) -> None:
    """nodes.py:1116-1132."""
    sps, ps = list(server_params), list(params)
    if hoststage.is_host(sps):  # the reference's CPU server: staged, folded on the device, written back in place
        with hoststage.staged([sps], [True], [True], [ps]) as ((dsps,), (dps,)):
            add_parameters(dsps, dps, ratio)
        return
    sps = _params(sps)
    if _fold(sps, [ps], [ratio], 2):
        return
    for sp, p in zip(sps, ps):  # (a float64, non-contiguous or spread model) per-tensor launches
        _weighted_sum_any(sp, [p], [ratio], 2)


def avg_parameters(server_params: Sequence[torch.Tensor], messages: Sequence[Mapping], size_aware: bool = False,
                   inertia: float = 0.0, key: str = "parameters") -> None:
    """nodes.py:1134-1163 (weights formed in double, message order preserved)."""
    assert 0.0 <= inertia < 1.0, "`inertia` should be in [0, 1)"
    if len(messages) == 0:
        return
    sps = list(server_params)
    if hoststage.is_host(sps):
        with hoststage.staged([sps], [True], [True], [m[key] for m in messages]) as ((dsps,), dmsgs):
            avg_parameters(dsps, [{key: d, "train_samples": m["train_samples"]} for m, d in zip(messages, dmsgs)],
                           size_aware, inertia, key)
        return
    total_samples = sum([m["train_samples"] for m in messages])
    ratios = [
        (m["train_samples"] / total_samples if size_aware else 1 / len(messages)) * (1 - inertia) for m in messages
    ]
    if _fold(_params(sps), messages, ratios, 0, inertia, key=key):
        return
    for j, sp in enumerate(_params(sps)):  # (a float64, non-contiguous or spread model) per-tensor launches
        _weighted_sum_any(sp, [m[key][j] for m in messages], ratios, 0, inertia)


def _gradients_on(dev: torch.device, messages: Sequence[Mapping]) -> List[torch.Tensor]:
    """Σ_m (ts_m / Σts) · g_m per tensor, folded on ``dev`` into one flat buffer's views."""
    total_samples = sum([m["train_samples"] for m in messages])
    weights = [m["train_samples"] / total_samples for m in messages]
    g0s = messages[0]["gradients"]
    dt = g0s[0].dtype
    flat = torch.empty(max(sum(g.numel() for g in g0s), 1), dtype=dt, device=dev)
    gs, off = [], 0
    for g in g0s:
        gs.append(flat[off:off + g.numel()].view(g.shape))
        off += g.numel()
    if all(g.dtype == dt for g in g0s) and _fold(gs, messages, weights, 1, key="gradients"):
        return gs
    gs = [torch.empty(g.shape, dtype=g.dtype, device=dev) for g in g0s]
    for j, g in enumerate(gs):
        codec.weighted_sum(g, [_on(m["gradients"][j], dev) for m in messages], weights, init_mode=1)
    return gs


def update_gradients(model_params: Sequence[torch.Tensor], messages: Sequence[Mapping]) -> Optional[List[torch.Tensor]]:
    """nodes.py:1165-1180: sets ``.grad`` of each model parameter to the sample-weighted gradient sum, on the model's
    device (a host-resident model gets host gradients, as the reference's ``.to(self.device)`` gives)."""
    if len(messages) == 0:
        return None
    assert all(["gradients" in m for m in messages]), "some clients have not sent gradients yet"
    model_params = list(model_params)
    if hoststage.is_host(model_params):
        dev = hoststage._device_for([m["gradients"] for m in messages])
        with torch.cuda.device(dev):
            dmsgs = hoststage.stage_messages([m["gradients"] for m in messages], dev, messages[0]["gradients"][0].dtype)
            dgs = _gradients_on(dev, [{"gradients": d, "train_samples": m["train_samples"]}
                                      for m, d in zip(messages, dmsgs)])
            grads = [g.to("cpu") for g in dgs]
    else:
        g0s = messages[0]["gradients"]
        devs = [mp.device if mp.device.type == "cuda" else g.device for mp, g in zip(model_params, g0s)]
        if len(set(devs)) == 1 and devs[0].type == "cuda":
            grads = _gradients_on(devs[0], messages)
        else:  # parameters spread over several HIP devices (the reference accepts any placement): per tensor, each
            # gradient folded on its own parameter's device
            total_samples = sum([m["train_samples"] for m in messages])
            weights = [m["train_samples"] / total_samples for m in messages]
            grads = []
            for j, d in enumerate(devs):
                if d.type != "cuda":
                    raise TypeError(f"update_gradients: parameter {j} and its gradients are not on a HIP device")
                g = torch.empty(g0s[j].shape, dtype=g0s[j].dtype, device=d)
                codec.weighted_sum(g, [_on(m["gradients"][j], d) for m in messages], weights, init_mode=1)
                grads.append(g)
    for mp, g in zip(model_params, grads):  # (every parameter, frozen ones too: nodes.py:1171-1172 sets them all)
        if isinstance(mp, torch.Tensor):
            mp.grad = g
    return grads


def _pair_fold(dev: torch.device, params: Sequence[torch.Tensor], messages: Sequence[Mapping], wp: Sequence[float],
               wg: Sequence[float], inertia: float):
    """flc_avg_and_gradients on ``dev``: the parameters folded in place, the gradients into one new flat buffer.
    Returns (gradient views, the flat buffer), or None (nothing launched) when a tensor is not a contiguous fp32
    tensor of ``dev``."""
    import ctypes

    fast = codec._pypair()
    if fast is not None:
        # one C call: every tensor checked in place (no per-tensor Python attribute reads, no ctypes tables); a
        # TypeError (a tensor the launch does not take) leaves everything untouched, as does None below
        flat = torch.empty(max(sum(p.numel() for p in params), 1), dtype=torch.float32, device=dev)
        grads, off = [], 0
        for p in params:
            grads.append(flat[off:off + p.numel()].view(p.shape))
            off += p.numel()
        try:
            fast(params, grads, messages, wp, wg, float(inertia))  # (on the current stream of the model's device)
            return grads, flat
        except TypeError:
            pass  # (messages on another device: moved below, as _on does)
    ok = lambda t: t.is_cuda and t.device == dev and t.dtype is torch.float32 and t.is_contiguous()  # noqa: E731
    if not all(ok(p) for p in params):
        return None
    T = len(params)
    psrc = [[_on(t, dev) for t in m["parameters"]] for m in messages]
    gsrc = [[_on(t, dev) for t in m["gradients"]] for m in messages]
    if any(len(r) != T or not all(ok(t) and t.numel() == p.numel() for t, p in zip(r, params))
           for r in psrc + gsrc):
        return None
    flat = torch.empty(max(sum(p.numel() for p in params), 1), dtype=torch.float32, device=dev)
    grads, off = [], 0
    for p in params:
        grads.append(flat[off:off + p.numel()].view(p.shape))
        off += p.numel()
    P = ctypes.c_void_p
    n = len(messages)
    _lib.call("flc_avg_and_gradients", (P * T)(*[p.data_ptr() for p in params]),
              (P * T)(*[g.data_ptr() for g in grads]),
              (P * (n * T))(*[t.data_ptr() for r in psrc for t in r]),
              (P * (n * T))(*[t.data_ptr() for r in gsrc for t in r]),
              (ctypes.c_float * n)(*wp), (ctypes.c_float * n)(*wg), n, (ctypes.c_int64 * T)(*[p.numel() for p in params]),
              T, float(inertia), codec._stream(dev))
    return grads, flat


def avg_parameters_and_gradients(model_params: Sequence[torch.Tensor], messages: Sequence[Mapping],
                                 size_aware: bool = False, inertia: float = 0.0) -> Optional[List[torch.Tensor]]:
    """``avg_parameters(size_aware, inertia)`` then ``update_gradients()`` (nodes.py:1134-1180) over the same messages
    in ONE launch (flc_avg_and_gradients) — the update of the variance-reduced servers (fedprox/_fedprox.py:163-167,
    fedpd/_fedpd.py:197-202, proxskip/_proxskip.py:212-216, pfedmac/_pfedmac.py:158-162).  Bit-identical to the two
    calls; a host-resident model is staged once (its messages and parameters in; the parameters and, in one copy, the
    gradients out).  Sets ``.grad`` of each parameter as update_gradients does and returns the gradients."""
    assert 0.0 <= inertia < 1.0, "`inertia` should be in [0, 1)"
    if len(messages) == 0:
        return None
    assert all(["gradients" in m for m in messages]), "some clients have not sent gradients yet"
    mps = list(model_params)
    total = sum([m["train_samples"] for m in messages])
    wp = [(m["train_samples"] / total if size_aware else 1 / len(messages)) * (1 - inertia) for m in messages]
    wg = [m["train_samples"] / total for m in messages]
    n = len(messages)
    if hoststage.is_host(mps):
        with hoststage.staged([mps], [True], [True], [m["parameters"] for m in messages]
                              + [m["gradients"] for m in messages]) as ((dps,), dm):
            dmsgs = [{"parameters": dm[i], "gradients": dm[n + i], "train_samples": m["train_samples"]}
                     for i, m in enumerate(messages)]
            dev = dps[0].device
            r = _pair_fold(dev, dps, dmsgs, wp, wg, inertia)
            if r is None:  # (a model the fused launch does not take: the two calls)
                avg_parameters(dps, dmsgs, size_aware, inertia)
                dg = _gradients_on(dev, dmsgs)
                flat = torch.cat([g.reshape(-1) for g in dg])
            else:
                dg, flat = r
            host = torch.empty(flat.numel(), dtype=flat.dtype, pin_memory=True)
            host.copy_(flat, non_blocking=True)  # one D2H copy, drained by the staging's synchronisation
        grads, off = [], 0
        for g in dg:
            grads.append(host[off:off + g.numel()].view(g.shape))
            off += g.numel()
    else:
        fast = codec._pypair()
        if fast is not None and mps and isinstance(mps[0], torch.Tensor) and mps[0].is_cuda:
            # one C call: the fold, the gradients' buffer and views, and every parameter's `.grad`; a TypeError (a
            # tensor the launch does not take, or messages elsewhere) leaves everything untouched
            try:
                return fast(mps, None, messages, wp, wg, float(inertia), True)[0]
            except TypeError:
                pass
        ps = _params(mps)
        r = _pair_fold(ps[0].device, ps, messages, wp, wg, inertia) if ps and ps[0].is_cuda else None
        if r is None:
            avg_parameters(mps, messages, size_aware, inertia)
            return update_gradients(mps, messages)
        grads = r[0]
    for mp, g in zip(mps, grads):
        if isinstance(mp, torch.Tensor):
            mp.grad = g
    return grads


def fedopt_update(model_params: Sequence[torch.Tensor], delta_parameters: Sequence[torch.Tensor],
                  v_parameters: Optional[Sequence[torch.Tensor]], messages: Sequence[Mapping], optimizer: str,
                  lr: float, betas: Sequence[float], tau: float) -> None:
    """_fedopt.py:196-265 (FedAvg: optimizer="avg", lr=1, betas=(0, 1))."""
    opt = optimizer.lower()
    if opt not in ("avg", "adagrad", "yogi", "adam"):
        raise ValueError(f"Unknown optimizer: {optimizer}")
    alpha = (1 - betas[0]) / len(messages) if len(messages) else 0.0
    model_params, delta_parameters = list(model_params), list(delta_parameters)
    vps = None if (v_parameters is None or opt == "avg") else list(v_parameters)
    recs = compressed.stacked_round(messages)  # a round of packed stacked records (the codec's call site)
    if hoststage.is_host(model_params):
        groups = [model_params, delta_parameters] + ([vps] if vps is not None else [])
        n = len(groups)
        msgs = [[d.record] for d in recs] if recs is not None else [m["delta_parameters"] for m in messages]
        with hoststage.staged(groups, [True] * n, [True] * n, msgs) as (dg, dm):
            if recs is not None and compressed.fold_records(
                    recs, [alpha] * len(recs), dg[1], _params(dg[0]), dg[2] if vps is not None else None, betas[0],
                    opt if vps is not None else "avg", lr, betas[1], tau):
                return
            fedopt_update(dg[0], dg[1], dg[2] if vps is not None else None,
                          [{"delta_parameters": m["delta_parameters"] if recs is not None else d}
                           for m, d in zip(messages, dm)], optimizer, lr, betas, tau)
        return
    # (the parameters as they are for the one-pass fold: its kernels write θ in place, outside autograd)
    if recs is not None and compressed.fold_records(recs, [alpha] * len(recs), delta_parameters, model_params, vps,
                                                    betas[0], opt if vps is not None else "avg", lr, betas[1], tau):
        return  # every record decoded, folded and the optimizer step applied in one pass
    ps = _params(model_params)
    if _fold(delta_parameters, messages, [alpha] * len(messages), 0, betas[0], key="delta_parameters",
             theta=ps, v=vps, opt=opt if vps is not None else "avg", lr=lr, beta2=betas[1], tau=tau):
        return  # the delta average and the optimizer step of every tensor in one launch
    for j, dp in enumerate(delta_parameters):
        _weighted_sum_any(dp, [m["delta_parameters"][j] for m in messages], [alpha] * len(messages), 0, betas[0])
    ps = _params(model_params)
    for j, (sp, dp) in enumerate(zip(ps, delta_parameters)):
        vp = None if (v_parameters is None or opt == "avg") else v_parameters[j]
        _contig_call(codec.fedopt_step, sp, dp, vp, opt if vp is not None else "avg", lr, betas[1], tau)


def scaffold_update(model_params: Sequence[torch.Tensor], control_variates: Sequence[torch.Tensor],
                    messages: Sequence[Mapping], lr: float, num_clients: int) -> None:
    """_scaffold.py:158-167.  The reference interleaves the two folds per message; they touch different tensors,
    so each tensor's fmaf chain (message order) is the same when folded in one launch per tensor."""
    if len(messages) == 0:
        raise ZeroDivisionError("division by zero")  # ratio_p = lr / len(messages) in the reference
    ratio_p = lr / len(messages)
    ratio_c = 1 / num_clients
    model_params, control_variates = list(model_params), list(control_variates)
    if hoststage.is_host(model_params):
        n = len(messages)
        with hoststage.staged([model_params, control_variates], [True, True], [True, True],
                              [m["parameters_delta"] for m in messages]
                              + [m["control_variates_delta"] for m in messages]) as ((dps, dcvs), dm):
            scaffold_update(dps, dcvs, [{"parameters_delta": a, "control_variates_delta": b}
                                        for a, b in zip(dm[:n], dm[n:])], lr, num_clients)
        return
    ps, cvs = _params(model_params), list(control_variates)
    if not _fold(ps, messages, [ratio_p] * len(messages), 2, key="parameters_delta"):
        for j, sp in enumerate(ps):
            _weighted_sum_any(sp, [m["parameters_delta"][j] for m in messages], [ratio_p] * len(messages), 2)
    if not _fold(cvs, messages, [ratio_c] * len(messages), 2, key="control_variates_delta"):
        for j, cv in enumerate(cvs):
            _weighted_sum_any(cv, [m["control_variates_delta"][j] for m in messages], [ratio_c] * len(messages), 2)


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
        center = list(cluster_centers[c]["center_model_params"])
        if hoststage.is_host(center):
            with hoststage.staged([center], [True], [True], [m["delta_parameters"] for m in ms]) as ((dc,), dm):
                for j, p in enumerate(dc):
                    _weighted_sum_any(p, [d[j] for d in dm], [1 / sizes[c]] * len(ms), 2)
            continue
        for j, p in enumerate(_params(center)):
            _weighted_sum_any(p, [m["delta_parameters"][j] for m in ms], [1 / sizes[c]] * len(ms), 2)
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
    model_params, y_params, x_til_params = list(model_params), list(y_params), list(x_til_params)
    if hoststage.is_host(model_params):
        with hoststage.staged([model_params, y_params, x_til_params], [True] * 3, [True] * 3,
                              [m["x_hat_delta"] for m in messages]) as ((dps, dys, dxs), dm):
            feddr_update(dps, dys, dxs, [{"x_hat_delta": d, "train_samples": m["train_samples"]}
                                         for m, d in zip(messages, dm)], alpha, eta, num_clients, reg_type)
        return
    coeff = eta * num_clients / (num_clients + 1)
    total = sum([m["train_samples"] for m in messages])
    weights = [m["train_samples"] / total for m in messages]
    for j, xt in enumerate(x_til_params):
        _weighted_sum_any(xt, [m["x_hat_delta"][j] for m in messages], weights, 2)
    cx, cy = coeff / eta, 1 / (num_clients + 1)
    if kind == "l1":
        prox, pc = _lib.FLC_PROX_L1, coeff
    elif kind == "l2squared":
        prox, pc = _lib.FLC_PROX_SCALE, 1 / (1 + 2 * coeff)
    else:
        prox, pc = _lib.FLC_PROX_NONE, 0.0
    ps = _params(model_params)
    for sp, yp, xt in zip(ps, y_params, x_til_params):
        _contig_call(codec.feddr_combine, sp, yp, xt, alpha, cx, cy, prox, pc)
    if kind == "l2":
        sq = 0.0
        for sp in ps:
            nrm = codec.quant_norm_f64(sp, 2) if sp.dtype == torch.float64 else codec.quant_norm(sp.reshape(1, -1), 2)
            sq += float(nrm.item()) ** 2
        norm = coeff * math.sqrt(sq)
        f = max(0, 1 - coeff / norm)
        for sp in ps:
            _weighted_sum_any(sp, [], [], 0, f)


def feddyn_update(model_params: Sequence[torch.Tensor], h_params: Sequence[torch.Tensor], messages: Sequence[Mapping],
                  mu: float, num_clients: int) -> None:
    """feddyn/_feddyn.py:172-184: ``h += -mu/N · (p_m − θ)`` for each message in order (θ still the old model), then
    ``avg_parameters()``; line 184 (``p = p.add(h, alpha=-1/mu)``) rebinds a local name and leaves the model as it is,
    so nothing follows.  Up to 16 messages: one launch for h and θ together (every operand read once); more: h in
    chained launches against the unchanged θ, then the chained average."""
    model_params, h_params = list(model_params), list(h_params)
    if len(messages) == 0:
        return  # (no h update; avg_parameters returns early)
    if hoststage.is_host(model_params):
        with hoststage.staged([model_params, h_params], [True, True], [True, True],
                              [m["parameters"] for m in messages]) as ((dps, dhs), dm):
            feddyn_update(dps, dhs, [{"parameters": d, "train_samples": m["train_samples"]}
                                     for m, d in zip(messages, dm)], mu, num_clients)
        return
    ps = _params(model_params)
    dev = ps[0].device
    alpha = -mu / num_clients
    w = [1 / len(messages)] * len(messages)
    cap = codec.MODEL_FOLD_MAX_SRC
    ps_ = codec._pysrv()
    if ps_ is not None and len(messages) <= cap:
        try:  # the common case in one C call: the messages already on the model's device
            ps_(ps, h_params, messages, "parameters", w, _lib.FLC_SRV_FEDDYN, 1, 0, 0.0, alpha)
            return
        except TypeError:
            pass  # messages elsewhere: moved below
    srcs = [[_on(t, dev) for t in m["parameters"]] for m in messages]
    if _srv_ok([ps, h_params] + srcs):
        if len(srcs) <= cap:
            codec.model_fold_server(ps, h_params, srcs, w, "feddyn", True, 0, 0.0, alpha)
            return
        for c0 in range(0, len(srcs), cap):
            codec.model_fold_server(ps, h_params, srcs[c0:c0 + cap], w[c0:c0 + cap], "feddyn", False, 0, 0.0, alpha)
    else:  # (a float64, non-contiguous or spread model) per-tensor launches
        for j, (p, h) in enumerate(zip(ps, h_params)):
            for m in messages:  # h = fmaf(alpha, fl(p_m - θ), h) in message order, θ still the old model
                d = _on(m["parameters"][j], p.device).clone().contiguous()
                _weighted_sum_any(d, [p], [-1.0], 2)  # fmaf(-1, θ, p_m) = fl(p_m - θ)
                _weighted_sum_any(h, [d], [alpha], 2)
    avg_parameters(ps, [{"parameters": s_, "train_samples": m["train_samples"]} for s_, m in zip(srcs, messages)])


def _srv_ok(groups) -> bool:
    """Every tensor of every group a contiguous fp32 tensor on the first one's device, sized as the first group
    (what flc_model_fold_server takes)."""
    if not groups or not groups[0]:
        return False
    dev = groups[0][0].device
    sizes = [t.numel() for t in groups[0]]
    return dev.type == "cuda" and all(
        len(g) == len(sizes) and all(t.device == dev and t.dtype is torch.float32 and t.is_contiguous()
                                     and t.numel() == k for t, k in zip(g, sizes)) for g in groups)


def _contig_call(fn, *ts, **kw) -> None:
    """fn(*ts, **kw) on contiguous stand-ins of non-contiguous tensors (an in-place kernel's operands), copied back
    afterwards; other arguments pass through."""
    cs = [t.contiguous() if isinstance(t, torch.Tensor) else t for t in ts]
    fn(*cs, **kw)
    for t, c in zip(ts, cs):
        if c is not t:
            t.copy_(c)


def _weighted_sum_any(dst: torch.Tensor, srcs, weights, init_mode: int, beta: float = 0.0) -> None:
    """codec.weighted_sum on a destination of any layout (a non-contiguous one through a contiguous copy)."""
    if dst.is_contiguous():
        codec.weighted_sum(dst, [_on(s_, dst.device) for s_ in srcs], weights, init_mode, beta)
        return
    tmp = dst.contiguous()
    codec.weighted_sum(tmp, [_on(s_, dst.device) for s_ in srcs], weights, init_mode, beta)
    dst.copy_(tmp)


def pfedme_update(model_params: Sequence[torch.Tensor], messages: Sequence[Mapping], beta: float) -> None:
    """pfedme/_pfedme.py:166-175: the previous model saved, ``avg_parameters()``, then
    ``θ = fl(θ · β) + (1 − β) · θ_prev`` (mul_ then add_ with alpha: one rounding, then one fma).  Up to 16 messages in
    one launch (θ_prev held in registers, never stored); more: θ saved, the chained average, then the blend."""
    model_params = list(model_params)
    if hoststage.is_host(model_params):
        with hoststage.staged([model_params], [True], [True], [m["parameters"] for m in messages]) as ((dps,), dm):
            pfedme_update(dps, [{"parameters": d, "train_samples": m["train_samples"]} for m, d in zip(messages, dm)],
                          beta)
        return
    ps = _params(model_params)
    dev = ps[0].device
    w = [1 / len(messages)] * len(messages) if messages else []
    ps_ = codec._pysrv()
    if ps_ is not None and len(messages) <= codec.MODEL_FOLD_MAX_SRC:
        try:  # the common case in one C call (no message: the blend of θ with itself, init 2)
            ps_(ps, ps, messages, "parameters", w, _lib.FLC_SRV_PFEDME, 1, 0 if messages else 2, 0.0, beta)
            return
        except TypeError:
            pass  # messages elsewhere: moved below
    srcs = [[_on(t, dev) for t in m["parameters"]] for m in messages]
    if _srv_ok([ps] + srcs):
        if len(srcs) <= codec.MODEL_FOLD_MAX_SRC:
            # (no message: avg_parameters returns before its mul_(inertia): the blend of θ with itself, init 2)
            codec.model_fold_server(ps, ps, srcs, w, "pfedme", True, 0 if srcs else 2, 0.0, beta)
            return
        saved = [p.detach().clone() for p in ps]
        avg_parameters(ps, [{"parameters": s_, "train_samples": m["train_samples"]} for s_, m in zip(srcs, messages)])
        codec.model_fold_server(ps, saved, [], [], "pfedme", False, 2, 0.0, beta)
    else:  # (a float64, non-contiguous or spread model) per-tensor launches
        saved = [p.detach().clone() for p in ps]
        avg_parameters(ps, [{"parameters": m["parameters"], "train_samples": m["train_samples"]} for m in messages])
        for p, pre in zip(ps, saved):  # θ = fmaf(1 - β, θ_prev, fl(θ · β)): mul_(beta).add_(prev, alpha=1 - beta)
            _weighted_sum_any(p, [pre], [1 - beta], 0, beta)


def _adopt(groups, messages_tensors=()) -> None:
    """The mixins own the server's tensors: a host-resident server's groups are adopted into one pinned buffer with a
    device mirror (hoststage.adopt), so each update stages them with one copy each way."""
    groups = [list(g) for g in groups if g is not None]
    if groups and hoststage.is_host(groups[0]):
        hoststage.adopt(groups, hoststage._device_for(messages_tensors))


class AggregationMixin:
    """Mix in before a reference ``Server`` subclass to run its aggregation on the device.

    The server model may live on a HIP device or in host memory (the reference's ``Server`` keeps it on the CPU,
    nodes.py:606): host tensors are staged to the device and written back in place, bit-identical either way.
    """

    def add_parameters(self, params, ratio: float) -> None:  # nodes.py:1116
        params = list(params)
        _adopt([list(self.model.parameters())], [params])
        add_parameters(self.model.parameters(), params, ratio)

    def avg_parameters(self, size_aware: bool = False, inertia: float = 0.0) -> None:  # nodes.py:1134
        _adopt([list(self.model.parameters())], [m["parameters"] for m in self._received_messages])
        avg_parameters(list(self.model.parameters()), self._received_messages, size_aware, inertia)

    def update_gradients(self) -> None:  # nodes.py:1165
        update_gradients(list(self.model.parameters()), self._received_messages)


class VRUpdateMixin:
    """Device ``update()`` for the reference's variance-reduced servers, whose update is ``avg_parameters`` then, with
    ``config.vr``, ``update_gradients``: FedProxServer (fedprox/_fedprox.py:163-167), ProxSkipServer
    (proxskip/_proxskip.py:212-216), FedPDServer (fedpd/_fedpd.py:197-202, which also records the round's client ids)
    and pFedMacServer (pfedmac/_pfedmac.py:158-162, inertia 1 - beta: set ``vr_inertia_from_beta = True``).  With
    ``vr`` the two run as ONE launch (:func:`avg_parameters_and_gradients`), on a device- or host-resident model."""

    vr_inertia_from_beta = False
    record_communicated_clients = False

    def update(self) -> None:
        if self.record_communicated_clients:  # fedpd/_fedpd.py:198
            self._communicated_clients = [m["client_id"] for m in self._received_messages]
        inertia = 1 - self.config.beta if self.vr_inertia_from_beta else 0.0
        mps = list(self.model.parameters())
        if hoststage.is_host(mps):
            keys = ["parameters"] + (["gradients"] if self.config.vr else [])
            _adopt([mps], [m[k] for m in self._received_messages for k in keys])
            mps = list(self.model.parameters())  # (the adopted tensors)
        if self.config.vr:
            avg_parameters_and_gradients(mps, self._received_messages, inertia=inertia)
        else:
            avg_parameters(mps, self._received_messages, inertia=inertia)


class FedProxUpdateMixin(VRUpdateMixin):
    """fedprox/_fedprox.py:163-167."""


class ProxSkipUpdateMixin(VRUpdateMixin):
    """proxskip/_proxskip.py:212-216."""


class FedPDUpdateMixin(VRUpdateMixin):
    """fedpd/_fedpd.py:197-202."""

    record_communicated_clients = True


class pFedMacUpdateMixin(VRUpdateMixin):  # noqa: N801 (the reference's class name: pFedMacServer)
    """pfedmac/_pfedmac.py:158-162."""

    vr_inertia_from_beta = True


class FedOptUpdateMixin:
    """Device ``update()`` for the reference's ``FedOptServer`` family (_fedopt.py:196-240), for a server model on a
    HIP device or in host memory."""

    def update(self) -> None:
        adaptive = self.v_parameters is not None and self.config.optimizer.lower() != "avg"
        recs = compressed.stacked_round(self._received_messages)  # (compressed messages: the fold reads the records)
        _adopt([list(self.model.parameters()), self.delta_parameters, self.v_parameters if adaptive else None],
               [[d.record] for d in recs] if recs is not None
               else [m["delta_parameters"] for m in self._received_messages])
        fedopt_update(list(self.model.parameters()), self.delta_parameters, self.v_parameters,
                      self._received_messages, self.config.optimizer, self.config.lr, self.config.betas,
                      self.config.tau)


class SCAFFOLDUpdateMixin:
    """Device ``update()`` for the reference's ``SCAFFOLDServer`` (_scaffold.py:158-167)."""

    def update(self) -> None:
        _adopt([list(self.model.parameters()), self._control_variates],
               [m["parameters_delta"] for m in self._received_messages])
        scaffold_update(list(self.model.parameters()), self._control_variates, self._received_messages,
                        self.config.lr, len(self._clients))


class IFCAUpdateMixin:
    """Device ``update()`` for the reference's ``IFCAServer`` (_ifca.py:167-195)."""

    def update(self) -> None:
        ifca_update(self._cluster_centers, self._received_messages, self.config.num_clusters)


class FedDRUpdateMixin:
    """Device ``update()`` for the reference's ``FedDRServer`` (_feddr.py:166-190)."""

    def update(self) -> None:
        _adopt([list(self.model.parameters()), self._y_parameters, self._x_til_parameters],
               [m["x_hat_delta"] for m in self._received_messages])
        feddr_update(list(self.model.parameters()), self._y_parameters, self._x_til_parameters,
                     self._received_messages, self.config.alpha, self.config.eta, self.config.num_clients,
                     self.config.reg_type)


class FedDynUpdateMixin:
    """Device ``update()`` for the reference's ``FedDynServer`` (feddyn/_feddyn.py:172-184), for a server model on a
    HIP device or in host memory (h kept next to the model)."""

    def update(self) -> None:
        _adopt([list(self.model.parameters()), self.h_params], [m["parameters"] for m in self._received_messages])
        feddyn_update(list(self.model.parameters()), self.h_params, self._received_messages, self.config.mu,
                      self.config.num_clients)


class pFedMeUpdateMixin:  # noqa: N801 (the reference's class name: pFedMeServer)
    """Device ``update()`` for the reference's ``pFedMeServer`` (pfedme/_pfedme.py:166-175)."""

    def update(self) -> None:
        _adopt([list(self.model.parameters())], [m["parameters"] for m in self._received_messages])
        pfedme_update(list(self.model.parameters()), self._received_messages, self.config.beta)
