"""One client shard per GPU and an RCCL reduce of the decoded, weighted client deltas.

The reference runs its clients one after another in one process and places client ``i`` on device
``i mod n_devices`` (nodes.py:706-713); the server then folds every client's delta into the global
update in message order (nodes.py:1165-1180, _fedopt.py:202-208).  Here each rank (one process per
GPU, ``torch.distributed`` over RCCL/xGMI) owns the clients ``i`` with ``i mod world == rank``:

1. each owned client's delta goes through the device codec and is decoded *into* the rank's partial
   sum with its weight fused in (``out = fmaf(w_i, decode_i, out)``, one pass, no dense temporary);
2. ONE ``reduce`` (sum, fp32) brings the partial sums to the root rank — the only exchange step of
   the round; an ``all_reduce`` is used instead when every replica needs the result.

Within a rank the fold is the reference's sequential fmaf chain; across ranks the summation order is
RCCL's, so the multi-GPU result matches the single-device one to ``1e-6 * sum_i |w_i d_i| + 1e-30``
(SURVEY §8(c)), not bit for bit.

The codec step is a callable so the same driver serves the stacked top-k codec, the dense
quantizers and identity; the default (:func:`stacked_decode_accumulate`) calls the HIP kernels.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence

import torch
import torch.distributed as dist

# codec step: (client delta, weight, accumulator, client index) -> None, accumulating in place
CodecStep = Callable[[torch.Tensor, float, torch.Tensor, int], None]


def client_shard(n_clients: int, world: int, rank: int) -> List[int]:
    """Clients owned by `rank`: the reference's round-robin device placement (nodes.py:706-713)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    return [i for i in range(n_clients) if i % world == rank]


def sample_weights(train_samples: Sequence[int]) -> List[float]:
    """w_i = ts_i / sum(ts), formed in double as nodes.py:1173-1180 forms them (rounded to fp32 by the kernels)."""
    total = sum(train_samples)
    if total <= 0:
        raise ValueError("total train_samples must be positive")
    return [ts / total for ts in train_samples]


def stacked_decode_accumulate(k: int, levels: int = 127, seed: int = 0, counter: int = 0) -> CodecStep:
    """Codec step of configs[3]/[4]: stacked top-k -> 8-bit dithering encode, weighted decode-accumulate."""
    from . import codec

    def step(delta: torch.Tensor, weight: float, acc: torch.Tensor, client: int) -> None:
        pkt = codec.stacked_encode(delta, k, levels, seed=seed + client, counter=counter)
        codec.stacked_decode(pkt, out=acc, weight=weight, accumulate=True)

    return step


def aggregate_round(deltas: Sequence[torch.Tensor], weights: Sequence[float], clients: Sequence[int],
                    step: CodecStep, out: Optional[torch.Tensor] = None, dst: Optional[int] = 0,
                    group=None) -> torch.Tensor:
    """Fold this rank's clients into a partial sum, then reduce over the process group.

    ``deltas[j]`` is the flat delta of client ``clients[j]`` (already on this rank's device) and
    ``weights[j]`` its weight.  ``dst`` = root rank for ``reduce`` (the result is valid there only), or
    ``None`` for an ``all_reduce``.  Without an initialised process group this is the single-device fold.
    """
    if len(deltas) != len(weights) or len(deltas) != len(clients):
        raise ValueError("deltas, weights and clients must have the same length")
    if out is None:
        if not deltas:
            raise ValueError("need `out` when this rank owns no client")
        out = torch.zeros_like(deltas[0])
    else:
        out.zero_()
    for d, w, c in zip(deltas, weights, clients):
        if d.shape != out.shape or d.dtype != torch.float32:
            raise ValueError("every delta must be a flat fp32 tensor shaped like `out`")
        step(d, float(w), out, c)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if dst is None:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        else:
            dist.reduce(out, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return out
