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

:func:`aggregate_round_wire` is SURVEY §8(e)'s sparse alternative for the stacked codec: every rank
encodes its clients into packed wire records (~5 bytes per kept entry + tile pointers: 1.35 MB per
25M-element client at k = 1 %, against 100 MB for a dense partial sum), ONE RCCL ``all_gather`` moves
the records, and the fold of ALL clients runs in client order in one pass (``flc_stacked_fold_wires``)
— so the result is bit-identical to the single-device sequential fold at every world size.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Protocol, Sequence

import torch
import torch.distributed as dist

# codec step: (client delta, weight, accumulator, client index) -> None, accumulating in place
CodecStep = Callable[[torch.Tensor, float, torch.Tensor, int], None]


def client_shard(n_clients: int, world: int, rank: int) -> List[int]:
    """Clients owned by `rank`: the reference's round-robin device placement (nodes.py:706-713)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world size {world}")
    return [i for i in range(n_clients) if i % world == rank]


def synthetic_client_delta(client: int, n: int, device: torch.device, seed: int = 5000,
                           scale: float = 1e-3) -> torch.Tensor:
    """Client ``client``'s synthetic flat delta (N(0, 1) * scale, n fp32 elements) from a generator keyed by the client
    id alone, so every rank that builds it holds the same values (the N > 1 self-check folds every client on rank 0)
    and distinct clients hold distinct deltas (no cache-resident repeats in the bench's configs[3] legs)."""
    g = torch.Generator(device=device).manual_seed(seed + client)
    return torch.randn(n, generator=g, device=device) * scale


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

    def many(deltas: Sequence[torch.Tensor], weights: Sequence[float], acc: torch.Tensor,
             clients: Sequence[int], accumulate: bool = True) -> None:
        """The rank's clients encoded into packed wire records (several: one batched launch), then all of them decoded
        into ``acc`` in client order in one pass (flc_stacked_fold_wires): the same packets and the same fmaf chain as
        one ``step`` per client.  ``accumulate=False``: ``acc`` is overwritten with the fold from +0 (what zeroing it
        first gives, without the zeroing pass and the read of ``acc``)."""
        n = acc.numel()
        recs = torch.empty(len(deltas), codec.stacked_wire_layout(n, k)[0], dtype=torch.uint8, device=acc.device)
        if len(deltas) == 1:
            codec.stacked_encode(deltas[0], k, levels, seed=seed + clients[0], counter=counter, wire=recs[0])
        else:
            codec.stacked_encode_batch(deltas, k, levels, seeds=[seed + c for c in clients], counter=counter,
                                       wires=recs)
        codec.stacked_fold_wires(recs, list(range(len(deltas))), [float(w) for w in weights], n, k, levels, out=acc,
                                 accumulate=accumulate)

    step.many = many
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
        out = torch.empty_like(deltas[0])
    for d in deltas:
        if d.shape != out.shape or d.dtype != torch.float32:
            raise ValueError("every delta must be a flat fp32 tensor shaped like `out`")
    many = getattr(step, "many", None)
    if many is not None and deltas:  # a codec that folds the rank's clients from +0 itself (records + one fold pass)
        many(deltas, weights, out, clients, accumulate=False)
    else:
        out.zero_()
        for d, w, c in zip(deltas, weights, clients):
            step(d, float(w), out, c)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        if dst is None:
            dist.all_reduce(out, op=dist.ReduceOp.SUM, group=group)
        else:
            dist.reduce(out, dst=dst, op=dist.ReduceOp.SUM, group=group)
    return out


class WireCodec(Protocol):
    """A codec whose per-client output is a fixed-size byte record (``stride`` bytes)."""

    stride: int

    def encode_into(self, delta: torch.Tensor, record: torch.Tensor, client: int) -> None:
        """Encode one client's flat delta into ``record`` (uint8, ``stride`` bytes)."""

    def fold(self, records: torch.Tensor, slots: Sequence[int], weights: Sequence[float],
             out: torch.Tensor) -> None:
        """``out = +0``, then ``out = fmaf(weights[c], decode(records[slots[c]]), out)`` for c in order."""


class StackedWireCodec:
    """The HIP stacked codec on packed wire records (flc_stacked_encode_tiled into the record,
    flc_stacked_fold_wires over the gathered records)."""

    def __init__(self, n: int, k: int, levels: int = 127, seed: int = 0, counter: int = 0):
        from . import codec

        self.n, self.k, self.levels, self.seed, self.counter = int(n), int(k), int(levels), int(seed), int(counter)
        self.stride = codec.stacked_wire_layout(self.n, self.k)[0]

    def encode_into(self, delta: torch.Tensor, record: torch.Tensor, client: int) -> None:
        from . import codec

        codec.stacked_encode(delta, self.k, self.levels, seed=self.seed + client, counter=self.counter, wire=record)

    def encode_many_into(self, deltas: Sequence[torch.Tensor], records: torch.Tensor, clients: Sequence[int]) -> None:
        """All of this rank's clients in one batched launch (flc_stacked_encode_batch): records[j] equals
        ``encode_into(deltas[j], records[j], clients[j])`` bit for bit."""
        from . import codec

        codec.stacked_encode_batch(deltas, self.k, self.levels, seeds=[self.seed + c for c in clients],
                                   counter=self.counter, wires=records[:len(deltas)])

    def fold(self, records: torch.Tensor, slots: Sequence[int], weights: Sequence[float],
             out: torch.Tensor) -> None:
        from . import codec

        codec.stacked_fold_wires(records, slots, weights, self.n, self.k, self.levels, out=out, accumulate=False)


def wire_slots(n_clients: int, world: int) -> List[int]:
    """Record index of client i in the all-gathered buffer: rank ``i % world``'s block of
    ``ceil(n_clients / world)`` records, position ``i // world`` in it."""
    per = -(-n_clients // world)
    return [(i % world) * per + i // world for i in range(n_clients)]


def aggregate_round_wire(deltas: Sequence[torch.Tensor], weights: Sequence[float], n_clients: int,
                         wire: WireCodec, out: Optional[torch.Tensor] = None, dst: Optional[int] = None,
                         group=None, device: Optional[torch.device] = None) -> torch.Tensor:
    """One round with the packed wire as the only exchange.

    ``deltas`` are this rank's clients in :func:`client_shard` order (client ``i`` with ``i % world == rank``);
    ``weights`` are the weights of ALL ``n_clients`` clients, in client order.  Each rank encodes its clients into
    its block of records, one ``all_gather`` collects every block, and the fold of all clients in client order runs
    on every rank (``dst`` = None) or on rank ``dst`` only (the result is valid there only).  The result equals the
    single-device fold of the same clients bit for bit, whatever the world size.
    """
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    mine = client_shard(n_clients, world, rank)
    if len(deltas) != len(mine):
        raise ValueError(f"rank {rank} owns clients {mine}: one delta each (got {len(deltas)})")
    if len(weights) != n_clients:
        raise ValueError("one weight per client (all clients, in client order)")
    dev = device if device is not None else (deltas[0].device if deltas else (out.device if out is not None else None))
    if dev is None:
        raise ValueError("need a device when this rank owns no client and no `out` is given")
    per = -(-n_clients // world)
    send = torch.empty(per, wire.stride, dtype=torch.uint8, device=dev)  # (padding bytes are never read)
    if len(deltas) > 1 and hasattr(wire, "encode_many_into"):  # the rank's clients in one launch
        wire.encode_many_into(deltas, send, mine)
    else:
        for j, d in enumerate(deltas):
            wire.encode_into(d, send[j], mine[j])
    if multi:
        recs = torch.empty(world * per, wire.stride, dtype=torch.uint8, device=dev)
        if dist.get_backend(group) == "gloo":  # (gloo: the list form)
            dist.all_gather(list(recs.chunk(world)), send, group=group)
        else:
            dist.all_gather_into_tensor(recs, send, group=group)
    else:
        recs = send
    if dst is None or rank == dst:
        if out is None:
            out = torch.empty(getattr(wire, "n"), dtype=torch.float32, device=dev)
        wire.fold(recs, wire_slots(n_clients, world), weights, out)
    return out


def round_parity(all_deltas: Sequence[torch.Tensor], weights: Sequence[float], wire: WireCodec, step: CodecStep,
                 dst: int = 0, group=None, device: Optional[torch.device] = None) -> Optional[dict]:
    """Self-check of one aggregation round across the process group (the bench's N > 1 evidence).

    Every rank runs the packed-wire round and the dense round (codec + RCCL reduce) over its own shard of the clients
    (``all_deltas[i]`` is client ``i``'s delta; each rank only reads its own clients' entries, ``dst`` reads them all).
    On ``dst`` the single-device fold of ALL clients is then computed locally with the codec step alone (one encode and
    one weighted decode-accumulate per client, in client order) and compared: the wire round must equal it bit for bit
    (the fold kernel is built to reproduce that chain exactly), the dense round within
    ``1e-6 * sum_i |w_i d_i| + 1e-30`` per element (RCCL's summation order across ranks; ``d_i`` the decoded client
    delta).  Returns the comparison on ``dst`` (None elsewhere)."""
    multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    world = dist.get_world_size(group) if multi else 1
    rank = dist.get_rank(group) if multi else 0
    n_clients = len(all_deltas)
    mine = client_shard(n_clients, world, rank)
    dev = device if device is not None else all_deltas[0].device
    wired = aggregate_round_wire([all_deltas[c] for c in mine], weights, n_clients, wire, dst=dst, group=group,
                                 device=dev)
    dense = aggregate_round([all_deltas[c] for c in mine], [weights[c] for c in mine], mine, step,
                            out=torch.empty(all_deltas[0].numel(), dtype=torch.float32, device=dev), dst=dst,
                            group=group)
    if rank != dst:
        return None
    # the single-device reference: the per-client chain (one encode + weighted decode-accumulate per client, in client
    # order) — the codec step itself, not the fold kernel the wire round uses; and sum_i |w_i d_i| from the same decodes
    single = torch.zeros_like(dense)
    bound = torch.zeros_like(dense)
    one = torch.empty_like(dense)
    for c in range(n_clients):
        step(all_deltas[c], float(weights[c]), single, c)
        one.zero_()
        step(all_deltas[c], float(weights[c]), one, c)
        bound.add_(one.abs())
    bound.mul_(1e-6).add_(1e-30)
    err = (dense - single).abs()
    wire_exact = bool(torch.equal(wired.view(torch.int32), single.view(torch.int32)))
    dense_ok = bool(torch.all(err <= bound).item())
    return {"clients": n_clients, "world": world, "wire_bit_exact": wire_exact, "dense_within_bound": dense_ok,
            "dense_max_err_over_bound": float((err / bound).max().item()), "ok": wire_exact and dense_ok}
