"""ORACLE — test infrastructure only.  Never imported by the product package (fl_sim_amd/).

One FedOpt round with the codec at its call site (the meaning tests/golden/gen_golden.py ``gen_round`` fixes from the
reference's own pieces), restated from this directory's codec and aggregation restatements:
FedOptClient.communicate's delta (``_fedopt.py:295-308`` → ``aggregation_ref.client_delta``), the flattened delta
through the compressors in order (``compressors.py:267-410`` → ``compressors_ref``), the decoded vector as the
message's ``delta_parameters``, then FedOptServer.update (``_fedopt.py:196-240`` → ``aggregation_ref.fedopt_update``).
The global ``random`` / ``np.random`` streams are consumed as the reference consumes them (the caller seeds them).
Pinned by ``tests/golden/round_codec.npz`` (tests/test_oracle_golden.py).
"""

from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import aggregation_ref as agg
from . import compressors_ref as ref


def compress(codec: str, x: np.ndarray) -> Tuple[np.ndarray, List[float], List[float]]:
    """(decoded vector, send per stage, input components per stage) of one client's flat delta."""
    D = x.shape[0]
    K = D // 100
    rnd = ref.python_random_stream()
    if codec in ("topk", "stacked10"):
        out, send = ref.topk(x, K)
        sends, ins = [float(send)], [float(D)]
        if codec == "stacked10":
            out, s2, _ = ref.standard_dithering(out, 10, np.inf, rnd)
            sends.append(float(s2))
            ins.append(float(D))
        return out, sends, ins
    if codec == "std8inf":
        out, send, _ = ref.standard_dithering(x, 8, np.inf, rnd)
        return out, [float(send)], [float(D)]
    if codec == "std4p2":
        out, send, _ = ref.standard_dithering(x, 4, 2, rnd)
        return out, [float(send)], [float(D)]
    if codec == "natural":
        out, send, _ = ref.natural(x, rnd)
        return out, [float(send)], [float(D)]
    if codec == "randk":
        S = np.arange(D)
        np.random.shuffle(S)  # the reference's own legacy-stream shuffle (compressors.py:285-287)
        out, send = ref.randk(x, K, D, S[:K])
        return out, [float(send)], [float(D)]
    raise ValueError(codec)


def fedopt_round(codec: str, theta: Sequence[torch.Tensor], delta: Sequence[torch.Tensor], v, locals_, sizes,
                 optimizer: str, lr: float, betas, tau: float):
    """Runs one round in place on ``theta`` / ``delta`` / ``v``; returns the per-client stats rows
    (sends of every stage, then inputs of every stage), as gen_round stores them."""
    msgs, stats = [], []
    for local, ts in zip(locals_, sizes):
        dps = agg.client_delta(local, [t.clone() for t in theta])
        flat = torch.cat([d.reshape(-1) for d in dps]).numpy()
        out, sends, ins = compress(codec, flat)
        out_t = torch.from_numpy(np.ascontiguousarray(out, dtype=np.float32))
        dec, off = [], 0
        for d in dps:
            dec.append(out_t[off:off + d.numel()].reshape(d.shape).clone())
            off += d.numel()
        msgs.append({"delta_parameters": dec, "train_samples": ts})
        stats.append(sends + ins)
    agg.fedopt_update(theta, delta, v, msgs, optimizer, lr, betas, tau)
    return stats
