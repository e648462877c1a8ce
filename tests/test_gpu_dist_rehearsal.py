"""The N > 1 aggregation round with its HIP parts on a GPU: 2 and 3 ranks sharing the one GPU of the test box.

RCCL refuses two ranks on one device, so the ranks talk over gloo (which stages device tensors through the host for
its all-gather and all-reduce); everything else is the multi-GPU path as the bench runs it (fl_sim_amd/dist.py):
each rank's clients encoded into packed wire records on the device (one batched launch for several), the records
all-gathered, the client-order fold of every record on the device (`aggregate_round_wire`); and the dense round —
the rank's clients folded into a device partial sum, then summed across ranks (`aggregate_round`, all-reduce form).
The wire round must equal the single-device sequential chain bit for bit at every world size, the dense round within
1e-6 * sum_i |w_i d_i| + 1e-30 (the cross-rank summation order), as `dist.round_parity` checks on the driver's
multi-GPU runs.  What this does not exercise is RCCL itself (covered at world size 1, tests/test_gpu_comm.py)."""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_CLIENTS, D, K, LEVELS = 7, 1_000_003, 10_000, 127
TS = [100 * (i + 1) for i in range(N_CLIENTS)]


def _deltas(dev):
    g = torch.Generator(device=dev).manual_seed(21)
    return [torch.randn(D, generator=g, device=dev) * 1e-3 for _ in range(N_CLIENTS)]


def _worker(rank, world, port, outdir):
    import torch.distributed as dist

    from fl_sim_amd import dist as fdist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        deltas = _deltas(dev)
        w = fdist.sample_weights(TS)
        mine = fdist.client_shard(N_CLIENTS, world, rank)
        wire = fdist.StackedWireCodec(D, K, LEVELS, seed=3, counter=1)
        step = fdist.stacked_decode_accumulate(K, LEVELS, seed=3, counter=1)
        wired = fdist.aggregate_round_wire([deltas[c] for c in mine], w, N_CLIENTS, wire, dst=None, device=dev)
        dense = fdist.aggregate_round([deltas[c] for c in mine], [w[c] for c in mine], mine, step,
                                      out=torch.empty(D, dtype=torch.float32, device=dev), dst=None)
        torch.cuda.synchronize()
        np.save(os.path.join(outdir, f"wire{rank}.npy"), wired.cpu().numpy())
        np.save(os.path.join(outdir, f"dense{rank}.npy"), dense.cpu().numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_wire_and_dense_rounds_across_ranks_on_the_gpu(world, tmp_path):
    import torch.multiprocessing as mp

    from fl_sim_amd import codec
    from fl_sim_amd import dist as fdist

    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, str(tmp_path))) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=100)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]

    # the single-device reference: one encode + weighted decode-accumulate per client, in client order
    dev = torch.device("cuda", 0)
    deltas = _deltas(dev)
    w = fdist.sample_weights(TS)
    step = fdist.stacked_decode_accumulate(K, LEVELS, seed=3, counter=1)
    single = torch.zeros(D, dtype=torch.float32, device=dev)
    bound = torch.zeros_like(single)
    one = torch.empty_like(single)
    for c in range(N_CLIENTS):
        step(deltas[c], float(w[c]), single, c)
        one.zero_()
        step(deltas[c], float(w[c]), one, c)
        bound.add_(one.abs())
    single, bound = single.cpu().numpy(), (bound * 1e-6 + 1e-30).cpu().numpy()
    assert np.count_nonzero(single) > N_CLIENTS * K // 2
    for r in range(world):
        wired = np.load(tmp_path / f"wire{r}.npy")
        dense = np.load(tmp_path / f"dense{r}.npy")
        assert np.array_equal(wired.view(np.uint32), single.view(np.uint32)), r
        assert np.all(np.abs(dense - single) <= bound), r
    assert sum(codec.topk_status_all().values()) == 0
