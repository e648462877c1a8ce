"""Packed-wire aggregation round (fl_sim_amd/dist.py: aggregate_round_wire) on CPU: gloo, world size 2 and 3.

The HIP wire codec is replaced by a CPU one built on the numpy oracle (tests may use the oracle as the checker):
the oracle's stacked encode packed into the library's record layout (flc_stacked_wire_layout, a host-only call),
and a CPU fold that decodes each record and applies torch CPU ``add_(alpha=w)`` (one fp32 fma per element,
SURVEY App. A.3).  Under test: the record layout round trip, the rank -> record-block mapping, the all-gather and
the client-order fold — the world-2/3 results must equal the single-process fold bit for bit.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fl_sim_amd import codec
from fl_sim_amd import dist as fdist
from oracle import compressors_ref as ref

N_CLIENTS, D, K, S = 5, 5000, 50, 127
TS = [100 * (i + 1) for i in range(N_CLIENTS)]


def _deltas():
    g = np.random.default_rng(11)
    return [torch.from_numpy((g.standard_normal(D) * 1e-3).astype(np.float32)) for _ in range(N_CLIENTS)]


class OracleWireCodec:
    def __init__(self, n, k, seed=0, counter=3):
        self.n, self.k, self.seed, self.counter = n, k, seed, counter
        self.stride, self.off = codec.stacked_wire_layout(n, k)

    def encode_into(self, delta, record, client):
        seed = self.seed + client
        _, kept, codes, pn = ref.stacked(delta.numpy(), self.k, S,
                                         lambda idx: ref.philox_uniforms_at(idx, seed, self.counter))
        order = np.argsort(kept)
        kept, codes = kept[order].astype(np.int32), codes[order]
        rec = record.numpy()
        rec[self.off["norm"]:self.off["norm"] + 4] = np.array([pn], dtype=np.float32).view(np.uint8)
        rec[self.off["idx"]:self.off["idx"] + 4 * self.k] = kept.view(np.uint8)
        rec[self.off["codes"]:self.off["codes"] + self.k] = codes
        nt = (self.n + codec.TILE - 1) // codec.TILE
        tiles = np.searchsorted(kept, np.arange(nt + 1) * codec.TILE).astype(np.int32)
        rec[self.off["tiles"]:self.off["tiles"] + 4 * (nt + 1)] = tiles.view(np.uint8)

    def decode(self, record):
        rec = record.numpy()
        pn = rec[self.off["norm"]:self.off["norm"] + 4].view(np.float32)[0]
        idx = rec[self.off["idx"]:self.off["idx"] + 4 * self.k].view(np.int32)
        codes = rec[self.off["codes"]:self.off["codes"] + self.k].astype(np.int64)
        lv = ref.standard_levels(S).astype(np.float32)[codes & 127]
        out = np.zeros(self.n, dtype=np.float32)
        out[idx] = np.where(codes >> 7, -lv, lv).astype(np.float32) * pn
        return torch.from_numpy(out)

    def fold(self, records, slots, weights, out):
        out.zero_()
        for s, w in zip(slots, weights):
            out.add_(self.decode(records[s]), alpha=float(np.float32(w)))


class BatchedOracleWireCodec(OracleWireCodec):
    """The same codec with the batched entry point (dist.StackedWireCodec.encode_many_into's form): a rank's clients
    in one call, records[j] for clients[j]."""

    calls = []

    def encode_many_into(self, deltas, records, clients):
        type(self).calls.append(tuple(clients))
        assert records.shape[0] >= len(deltas)
        for j, (d, c) in enumerate(zip(deltas, clients)):
            self.encode_into(d, records[j], c)


def _single(deltas, w):
    wc = OracleWireCodec(D, K)
    return fdist.aggregate_round_wire(deltas, w, N_CLIENTS, wc, device=torch.device("cpu"))


def _worker(rank, world, port, q, batched=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        deltas = _deltas()
        w = fdist.sample_weights(TS)
        mine = fdist.client_shard(N_CLIENTS, world, rank)
        wc = BatchedOracleWireCodec(D, K) if batched else OracleWireCodec(D, K)
        res = fdist.aggregate_round_wire([deltas[c] for c in mine], w, N_CLIENTS, wc, device=torch.device("cpu"))
        q.put((rank, res.numpy().copy()))
        res0 = fdist.aggregate_round_wire([deltas[c] for c in mine], w, N_CLIENTS, wc, dst=0,
                                          device=torch.device("cpu"))
        q.put((rank + 100, None if res0 is None else res0.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_wire_layout_host_call():
    stride, off = codec.stacked_wire_layout(D, K)
    assert stride % 256 == 0 and off["norm"] == 0 and off["idx"] == 16
    assert off["codes"] >= off["idx"] + 4 * K and off["codes"] % 16 == 0
    assert off["tiles"] >= off["codes"] + max(K, 16) and off["tiles"] % 16 == 0
    assert stride >= off["tiles"] + 4 * ((D + codec.TILE - 1) // codec.TILE + 1)
    with pytest.raises(ValueError):
        codec.stacked_wire_layout(0, 1)


def test_wire_slots_mapping():
    assert fdist.wire_slots(5, 1) == [0, 1, 2, 3, 4]
    assert fdist.wire_slots(5, 2) == [0, 3, 1, 4, 2]
    for n, w in ((8, 3), (9, 4), (3, 8)):
        sl = fdist.wire_slots(n, w)
        per = -(-n // w)
        assert len(set(sl)) == n and max(sl) < w * per
        for i, s in enumerate(sl):  # client i sits in rank (i % w)'s block at position i // w
            assert s // per == i % w and s % per == i // w


def test_single_process_wire_round_is_the_sequential_fold():
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    got = _single(deltas, w).numpy()
    exp = torch.zeros(D, dtype=torch.float32)
    for i, (d, wi) in enumerate(zip(deltas, w)):
        out, *_ = ref.stacked(d.numpy(), K, S, lambda idx, i=i: ref.philox_uniforms_at(idx, i, 3))
        exp.add_(torch.from_numpy(out), alpha=float(np.float32(wi)))
    assert np.array_equal(got.view(np.uint32), exp.numpy().view(np.uint32))


def test_single_process_batched_codec_gets_all_clients_in_one_call():
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    BatchedOracleWireCodec.calls = []
    got = fdist.aggregate_round_wire(deltas, w, N_CLIENTS, BatchedOracleWireCodec(D, K), device=torch.device("cpu"))
    assert BatchedOracleWireCodec.calls == [tuple(range(N_CLIENTS))]
    assert np.array_equal(got.numpy().view(np.uint32), _single(deltas, w).numpy().view(np.uint32))


def test_wire_round_rejects_wrong_shard():
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    with pytest.raises(ValueError):
        fdist.aggregate_round_wire(deltas[:2], w, N_CLIENTS, OracleWireCodec(D, K), device=torch.device("cpu"))
    with pytest.raises(ValueError):
        fdist.aggregate_round_wire(deltas, w[:2], N_CLIENTS, OracleWireCodec(D, K), device=torch.device("cpu"))


@pytest.mark.parametrize("world,batched", [(2, False), (3, False), (2, True)])
def test_gloo_wire_round_is_bit_identical_to_single_process(world, batched):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, batched)) for r in range(world)]
    for p in procs:
        p.start()
    items = dict(q.get(timeout=180) for _ in range(2 * world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    single = _single(_deltas(), fdist.sample_weights(TS)).numpy()
    for r in range(world):  # every rank folds every client in client order: exact, not a tolerance
        assert np.array_equal(items[r].view(np.uint32), single.view(np.uint32))
    assert np.array_equal(items[100].view(np.uint32), single.view(np.uint32))
    assert all(items[100 + r] is None for r in range(1, world))


def _oracle_dense_step(wc):
    def step(delta, w, acc, client):  # encode, decode, fold with add_(alpha): the dense round's codec step on CPU
        rec = torch.zeros(wc.stride, dtype=torch.uint8)
        wc.encode_into(delta, rec, client)
        acc.add_(wc.decode(rec), alpha=float(np.float32(w)))

    return step


class _BrokenWireCodec(OracleWireCodec):
    """A broken fold (the last client left out) — round_parity must flag it."""

    def fold(self, records, slots, weights, out):
        super().fold(records, list(slots)[:-1], list(weights)[:-1], out)


def _parity_worker(rank, world, port, q, broken):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        wc = (_BrokenWireCodec if broken else OracleWireCodec)(D, K)
        res = fdist.round_parity(_deltas(), fdist.sample_weights(TS), wc, _oracle_dense_step(OracleWireCodec(D, K)),
                                 dst=0, device=torch.device("cpu"))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,broken", [(2, False), (3, False), (2, True)])
def test_gloo_round_parity_self_check(world, broken):
    """bench.py's N > 1 self-check (dist.round_parity) rehearsed on CPU: the wire round is bit-identical to the local
    single-device per-client chain, the dense round (gloo reduce) within 1e-6 * sum|w d| + 1e-30; a broken fold is caught."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_parity_worker, args=(r, world, port, q, broken)) for r in range(world)]
    for p in procs:
        p.start()
    items = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(items[r] is None for r in range(1, world))
    res = items[0]
    assert res["clients"] == N_CLIENTS and res["world"] == world and res["dense_within_bound"]
    assert res["wire_bit_exact"] is (not broken) and res["ok"] is (not broken)


def _distinct_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cpu = torch.device("cpu")
        deltas = [fdist.synthetic_client_delta(c, D, cpu) for c in range(N_CLIENTS)]
        sums = torch.tensor([float(d.double().sum()) for d in deltas], dtype=torch.float64)
        got = [torch.zeros_like(sums) for _ in range(world)]
        dist.all_gather(got, sums)
        res = fdist.round_parity(deltas, fdist.sample_weights(TS), OracleWireCodec(D, K),
                                 _oracle_dense_step(OracleWireCodec(D, K)), dst=0, device=cpu)
        q.put((rank, (res, [g.tolist() for g in got])))
    finally:
        dist.destroy_process_group()


def test_gloo_round_parity_with_distinct_synthetic_clients():
    """bench.py's configs[3] legs and N > 1 parity round use distinct client deltas (dist.synthetic_client_delta, a
    generator keyed by the client id): every rank builds the same deltas, the clients differ from each other, and the
    self-check passes on them (gloo world 2)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_distinct_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    items = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res, sums = items[0]
    assert sums[0] == sums[1], "every rank holds the same client deltas"
    assert len(set(sums[0])) == N_CLIENTS, "the clients' deltas are distinct"
    assert res["ok"] and res["wire_bit_exact"] and res["clients"] == N_CLIENTS
    assert items[1][0] is None
