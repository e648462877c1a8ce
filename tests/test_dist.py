"""Multi-process aggregation driver (fl_sim_amd/dist.py) on CPU: gloo, world size 2.

The device codec step is replaced by the numpy oracle's top-k (tests may use the oracle as the
checker); what is under test here is the sharding, the in-rank fmaf fold and the reduce.  The GPU
path of the same driver (RCCL, HIP codec step) runs in bench.py's configs[3] line at N > 1.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fl_sim_amd import dist as fdist
from oracle import compressors_ref as ref

N_CLIENTS, D, K = 5, 4099, 41
TS = [100 * (i + 1) for i in range(N_CLIENTS)]  # configs[3]: ts_i = 100 (i + 1)


def _deltas():
    g = np.random.default_rng(7)
    return [torch.from_numpy((g.standard_normal(D) * 1e-3).astype(np.float32)) for _ in range(N_CLIENTS)]


def _cpu_topk_step(delta, w, acc, client):
    # torch CPU add_(alpha) is one fp32 fma per element, the kernels' fold
    acc.add_(torch.from_numpy(ref.topk(delta.numpy(), K)[0]), alpha=w)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        deltas = _deltas()
        w = fdist.sample_weights(TS)
        mine = fdist.client_shard(N_CLIENTS, world, rank)
        out = torch.empty(D, dtype=torch.float32)
        res = fdist.aggregate_round([deltas[c] for c in mine], [w[c] for c in mine], mine, _cpu_topk_step,
                                    out=out, dst=0)
        if rank == 0:
            q.put(res.numpy().copy())
        res2 = fdist.aggregate_round([deltas[c] for c in mine], [w[c] for c in mine], mine, _cpu_topk_step,
                                     out=torch.empty(D, dtype=torch.float32), dst=None)
        q.put((rank, res2.numpy().copy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_client_shard_round_robin():
    assert fdist.client_shard(5, 2, 0) == [0, 2, 4]
    assert fdist.client_shard(5, 2, 1) == [1, 3]
    assert sorted(sum((fdist.client_shard(10, 4, r) for r in range(4)), [])) == list(range(10))
    with pytest.raises(ValueError):
        fdist.client_shard(3, 2, 2)


def test_sample_weights_double():
    w = fdist.sample_weights(TS)
    assert w == [t / sum(TS) for t in TS]
    with pytest.raises(ValueError):
        fdist.sample_weights([0, 0])


def test_single_process_fold_is_sequential_fmaf():
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    got = fdist.aggregate_round(deltas, w, list(range(N_CLIENTS)), _cpu_topk_step)
    exp = np.zeros(D, dtype=np.float32)
    for d, wi in zip(deltas, w):
        exp = (np.float64(np.float32(wi)) * ref.topk(d.numpy(), K)[0].astype(np.float64) + exp).astype(np.float32)
    assert np.array_equal(got.numpy().view(np.uint32), exp.view(np.uint32))


def test_gloo_world2_reduce_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    items = [q.get(timeout=120) for _ in range(3)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reduced = [it for it in items if not isinstance(it, tuple)][0]
    allred = {it[0]: it[1] for it in items if isinstance(it, tuple)}
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    single = fdist.aggregate_round(deltas, w, list(range(N_CLIENTS)), _cpu_topk_step).numpy()
    scale = sum(abs(wi) * np.abs(ref.topk(d.numpy(), K)[0]).astype(np.float64) for d, wi in zip(deltas, w))
    tol = 1e-6 * scale + 1e-30  # cross-rank summation order is the collective's
    assert np.all(np.abs(reduced.astype(np.float64) - single) <= tol)
    assert np.array_equal(allred[0], allred[1])
    assert np.all(np.abs(allred[0].astype(np.float64) - single) <= tol)


def test_fold_dispatches_to_a_batched_codec_step():
    """A codec step with a ``many`` attribute (the batched encoders' form, dist.stacked_decode_accumulate) gets the
    rank's clients in one call, in client order, and folds them from +0 itself (``accumulate=False``: no zeroing pass
    and no read of the accumulator) — for a single client too.  The fold equals the per-client one."""
    calls = []

    def step(delta, w, acc, client):
        calls.append(("one", client))
        _cpu_topk_step(delta, w, acc, client)

    def many(deltas, weights, acc, clients, accumulate=True):
        calls.append(("many", tuple(clients), accumulate))
        if not accumulate:
            acc.zero_()
        for d, w, c in zip(deltas, weights, clients):
            _cpu_topk_step(d, float(w), acc, c)

    step.many = many
    deltas = _deltas()
    w = fdist.sample_weights(TS)
    got = fdist.aggregate_round(deltas, w, list(range(N_CLIENTS)), step, out=torch.full((D,), 7.0))
    assert calls == [("many", tuple(range(N_CLIENTS)), False)]
    ref_out = fdist.aggregate_round(deltas, w, list(range(N_CLIENTS)), _cpu_topk_step)
    assert np.array_equal(got.numpy().view(np.uint32), ref_out.numpy().view(np.uint32))
    calls.clear()
    fdist.aggregate_round(deltas[:1], w[:1], [0], step)
    assert calls == [("many", (0,), False)]
