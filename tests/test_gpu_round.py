"""GPU parity of the codec's call site (fl_sim_amd/compressed.py): a FedOpt round of 10 clients, each sending its
delta through the drop-in compressors from the reference's FedOptClient.communicate position, then the server's
update — against the reference's own round (tests/golden/round_codec.npz, gen_golden.py ``gen_round``: the
reference's communicate -> compressVector -> FedOptServer.update), bit for bit, on a device-resident and a
host-resident (nodes.py:606) server, with every compressor's send statistics and both global streams in lock-step.

The stacked pipeline's messages carry packed wire records and the server folds them in one flc_fedopt_fold_records
pass; the other compressors' messages carry the decoded delta.  Also: the fused fold against the dense decode + fold
(chained record and tensor groups, misaligned tensors, every optimiser), and philox mode against the oracle."""

import math
import random
import types

import numpy as np
import pytest
import torch

from tests import golden_cases as gc
from tests.golden.gen_golden import (CONFIG1_SHAPES, ROUND_CLIENTS, ROUND_CODECS, ROUND_OPTS, SMALL_SHAPES,
                                     round_inputs, round_seed)

pytestmark = pytest.mark.gpu


def _fields(case):
    z = np.load(f"{gc.GOLDEN}/round_codec.npz", allow_pickle=False)
    out = {}
    for k in z.files:
        parts = k.split("|")
        if parts[0] != case:
            continue
        if len(parts) == 3:
            out.setdefault(parts[1], {})[parts[2]] = z[k]
        else:
            out[parts[1]] = z[k]
    return out


def _flat(ts):
    return torch.cat([t.detach().reshape(-1).cpu() for t in ts]).numpy()


def _same(rec, field, ts):
    a = _flat(ts)
    if "out" in rec[field]:
        return gc.same_bits(a, rec[field]["out"])
    return gc.sha(a) == str(rec[field]["sha"])


def make_compressors(codec, D, rng="compat", seed=0):
    from fl_sim_amd import Compressor

    def std(L, p):
        c = Compressor(rng=rng, seed=seed)
        nc = Compressor("norm")
        nc.makeIdenticalCompressor()
        c.makeStandardDitheringFP32(L, nc, p)
        return c

    if codec in ("topk", "stacked10"):
        c = Compressor(rng=rng, seed=seed)
        c.makeTopKCompressor(D // 100, D)
        return [c] + ([std(10, np.inf)] if codec == "stacked10" else [])
    if codec == "std8inf":
        return [std(8, np.inf)]
    if codec == "std4p2":
        return [std(4, 2)]
    if codec == "natural":
        c = Compressor(rng=rng, seed=seed)
        c.makeNaturalCompressorFP32()
        return [c]
    if codec == "randk":
        c = Compressor(rng=rng, seed=seed)
        c.makeRandKCompressor(D // 100, D)
        return [c]
    raise ValueError(codec)


def build_round(shapes, opt, server_device, n_clients=ROUND_CLIENTS):
    """(server, clients) objects with the mixins, holding round_inputs' tensors; the clients' models on cuda:0."""
    from fl_sim_amd.aggregation import FedOptUpdateMixin
    from fl_sim_amd.compressed import CompressedFedOptClientMixin

    theta, delta, v, locals_, sizes = round_inputs(shapes, opt, n_clients)

    class Server(FedOptUpdateMixin):
        pass

    class Client(CompressedFedOptClientMixin):
        pass

    s = Server()
    s.model = torch.nn.Module()
    for i, t in enumerate(theta):
        s.model.register_parameter(f"p{i}", torch.nn.Parameter(t.clone().to(server_device)))
    s.delta_parameters = [t.clone().to(server_device) for t in delta]
    s.v_parameters = None if v is None else [t.clone().to(server_device) for t in v]
    s.config = types.SimpleNamespace(optimizer=opt, **ROUND_OPTS[opt])
    s._received_messages = []
    clients = []
    for i, local in enumerate(locals_):
        c = Client()
        c.client_id, c._metrics = i, {}
        c.train_loader = types.SimpleNamespace(dataset=list(range(sizes[i])))
        c.model = torch.nn.Module()
        for j, t in enumerate(local):
            c.model.register_parameter(f"p{j}", torch.nn.Parameter(t.clone().cuda()))
        c._cached_parameters = [t.clone().cuda() for t in theta]
        clients.append(c)
    return s, clients


@pytest.mark.parametrize("server", ["device", "host"])
@pytest.mark.parametrize("tag", ["small", "config1"])
@pytest.mark.parametrize("opt", list(ROUND_OPTS))
@pytest.mark.parametrize("codec", ROUND_CODECS)
def test_compressed_round_matches_reference(codec, opt, tag, server):
    from fl_sim_amd.compressed import CompressedDelta

    shapes = SMALL_SHAPES if tag == "small" else CONFIG1_SHAPES
    rec = _fields(f"round_{codec}_{opt}_{tag}")
    s, clients = build_round(shapes, opt, "cuda" if server == "device" else "cpu")
    D = sum(int(np.prod(sh)) for sh in shapes)
    stats = []
    gc.seed_all(round_seed(codec, opt, tag))
    for c in clients:  # nodes.py:944-971: the clients of a round, one after the other
        c.compressors = make_compressors(codec, D)
        c.communicate(s)
        stats.append([float(x.last_need_to_send_advance) for x in c.compressors]
                     + [float(x.total_input_components) for x in c.compressors])
    assert random.random() == float(rec["next_random"])
    assert np.random.random_sample() == float(rec["next_np"])
    assert np.array_equal(np.array(stats, dtype=np.float64), rec["stats"])
    msgs = s._received_messages
    assert all(isinstance(m["delta_parameters"], CompressedDelta) for m in msgs)
    if codec == "stacked10":  # the wire, not the dense delta: 5 B per kept entry + tile pointers
        assert all(m["delta_parameters"].kind == "stacked" and m["delta_parameters"].nbytes < D for m in msgs)
    s.update()
    assert all(m["delta_parameters"]._flat is None for m in msgs) or codec != "stacked10"  # (never decoded densely)
    assert _same(rec, "delta", s.delta_parameters)  # the fold: bit for bit, every optimiser
    if opt == "avg":
        assert _same(rec, "theta", list(s.model.parameters()))
    else:
        _check_adaptive_tail(codec, opt, tag, shapes, s)
    if server == "host":
        assert all(p.is_cpu for p in s.model.parameters())


def _check_adaptive_tail(codec, opt, tag, shapes, s):
    """The adaptive optimisers' tail against the oracle's round (oracle/round_ref.py, pinned to the same fixture on
    CPU by tests/test_oracle_round.py), with the tolerance of test_gpu_aggregation.test_fedopt_update_matches_reference:
    torch's CPU scalar tail loop may contract v's update to an fma (v: 1 ulp) and its vectorised sqrt is not correctly
    rounded (θ: 1e-6 of the update + 1 ulp), where the kernels round every step as IEEE prescribes."""
    from oracle import round_ref

    theta, delta, v, locals_, sizes = round_inputs(shapes, opt)
    theta0 = _flat(theta)
    cfg = ROUND_OPTS[opt]
    gc.seed_all(round_seed(codec, opt, tag))
    round_ref.fedopt_round(codec, theta, delta, v, locals_, sizes, opt, cfg["lr"], cfg["betas"], cfg["tau"])
    assert gc.same_bits(_flat(s.delta_parameters), _flat(delta))
    exp_v, got_v = _flat(v), _flat(s.v_parameters)
    ulp_v = np.abs(exp_v.view(np.int32).astype(np.int64) - got_v.view(np.int32).astype(np.int64))
    assert ulp_v.max() <= 1 and (ulp_v > 0).mean() < 0.01
    exp_t, got_t = _flat(theta), _flat(list(s.model.parameters()))
    upd = np.abs(exp_t.astype(np.float64) - theta0)
    err = np.abs(exp_t.astype(np.float64) - got_t.astype(np.float64))
    assert np.all(err <= 1e-6 * upd + np.spacing(np.abs(exp_t)))


def test_compressed_delta_reads_as_the_decoded_tensors():
    """A server that is not the mixin (the reference's own update) reads the message's delta as a list of tensors: the
    record's dense decode, in the model's shapes."""
    from fl_sim_amd import codec
    from fl_sim_amd.compressed import compress_delta

    shapes = CONFIG1_SHAPES
    theta, _, _, locals_, _ = round_inputs(shapes, "avg", 1)
    D = sum(int(np.prod(sh)) for sh in shapes)
    gc.seed_all(3)
    d = compress_delta([t.cuda() for t in locals_[0]], [t.cuda() for t in theta], make_compressors("stacked10", D))
    dense = codec.stacked_decode(codec.wire_packet(d.record, d.n, d.k, d.levels)).cpu()
    assert len(d) == len(shapes) and [tuple(t.shape) for t in d] == [tuple(s) for s in shapes]
    got = torch.cat([t.reshape(-1).cpu() for t in d])
    assert gc.same_bits(got.numpy(), dense.numpy())


def _dense_reference_fold(recs, weights, delta, theta, v, beta0, opt, lr, beta2, tau):
    """The same update through the dense path: every record decoded, then flc_model_fold (init 0) with the step."""
    from fl_sim_amd import codec
    from fl_sim_amd.aggregation import fedopt_update

    msgs = []
    for r in recs:
        flat = codec.stacked_decode(codec.wire_packet(r.record, r.n, r.k, r.levels))
        off, ts = 0, []
        for t in delta:
            ts.append(flat[off:off + t.numel()].view(t.shape))
            off += t.numel()
        msgs.append({"delta_parameters": ts})
    n = len(msgs)
    betas = (beta0, beta2)
    # fedopt_update forms alpha = (1 - beta0) / n itself: check the caller's weights are that
    assert all(w == np.float32((1 - beta0) / n) for w in weights)
    fedopt_update(theta, delta, v, msgs, opt, lr, betas, tau)


@pytest.mark.parametrize("opt", ["avg", "adagrad", "yogi", "adam"])
@pytest.mark.parametrize("sizes,n_clients", [([400, 16, 12800, 32, 401408, 256, 2560, 10], 10),
                                             ([3, 1, 1027, 5, 0, 2049, 7, 4093] + list(range(1, 30)), 70),
                                             ([5, 2], 1), ([1000003], 3)])
def test_fold_records_matches_dense_decode_and_fold(opt, sizes, n_clients):
    """flc_fedopt_fold_records (one pass per 64 records and 16 tensors) against decoding every record and folding
    through flc_model_fold: bit for bit, every optimiser, odd / empty / misaligned tensors, > 64 clients."""
    from fl_sim_amd import codec
    from fl_sim_amd.compressed import CompressedDelta, fold_records

    n = sum(sizes)
    k = max(n // 100, 1)
    g = torch.Generator(device="cuda").manual_seed(n + n_clients)
    recs = []
    for c in range(n_clients):
        x = torch.randn(n, generator=g, device="cuda") * 1e-3
        x[torch.rand(n, generator=g, device="cuda") < 0.05] = 0.0
        stride, _ = codec.stacked_wire_layout(n, k)
        rec = torch.empty(stride, dtype=torch.uint8, device="cuda")
        codec.stacked_encode(x, k, 127, seed=c, counter=5, wire=rec)
        recs.append(CompressedDelta([torch.Size([n])], x.device, n, record=rec, k=k, levels=127))

    def state():
        base = torch.randn(3 * n + 8, generator=g, device="cuda") * 1e-2
        # misaligned views (one element in), then each group cut into the model's tensors
        out = []
        for gi in range(3):
            flat = base[1 + gi * n: 1 + (gi + 1) * n]
            ts, off = [], 0
            for s in sizes:
                ts.append(flat[off:off + s])
                off += s
            out.append(ts)
        theta, delta, v = out
        v = [t.abs() + 1e-6 for t in v]
        return theta, delta, v

    theta, delta, v = state()
    a_t, a_d, a_v = [t.clone() for t in theta], [t.clone() for t in delta], [t.clone() for t in v]
    beta0, lr, beta2, tau = (0.0, 1.0, 1.0, 1.0) if opt == "avg" else (0.9, 0.01, 0.99, 1e-3)
    w = [float(np.float32((1 - beta0) / n_clients))] * n_clients
    vv = None if opt == "avg" else a_v
    assert fold_records(recs, w, a_d, a_t, vv, beta0, opt, lr, beta2, tau)
    b_t, b_d, b_v = [t.clone() for t in theta], [t.clone() for t in delta], [t.clone() for t in v]
    _dense_reference_fold(recs, w, b_d, b_t, None if opt == "avg" else b_v, beta0, opt, lr, beta2, tau)
    for a, b in zip(a_t + a_d + a_v, b_t + b_d + b_v):
        assert gc.same_bits(a.cpu().numpy(), b.cpu().numpy())


def test_stacked_round_philox_matches_oracle():
    """Philox mode: the client's delta formed inside the encoder's read (flc_stacked_encode_delta into the record),
    the dithering stage's send count resolved from the device; the server's fused fold against the oracle's stacked
    codec (per-client Philox uniforms) and the reference's update restated (oracle/aggregation_ref)."""
    from oracle import aggregation_ref as agg_ref
    from oracle import compressors_ref as ref

    shapes = CONFIG1_SHAPES
    s, clients = build_round(shapes, "adam", "cuda")
    theta, delta, v, locals_, sizes = round_inputs(shapes, "adam")
    D = sum(int(np.prod(sh)) for sh in shapes)
    K = D // 100
    msgs = []
    for i, c in enumerate(clients):
        c.compressors = make_compressors("stacked10", D, rng="philox", seed=100 + i)
        st = c.compressors[1].philox.seed, c.compressors[1].philox.counter
        c.communicate(s)
        x = torch.cat([d.reshape(-1) for d in agg_ref.client_delta(locals_[i], theta)]).numpy()
        out, kept, _, _ = ref.stacked(x, K, 10, lambda idx, st=st: ref.philox_uniforms_at(idx, st[0], st[1]))
        off, ts = 0, []
        for sh in shapes:
            m = int(np.prod(sh))
            ts.append(torch.from_numpy(out[off:off + m].copy()).view(sh))
            off += m
        msgs.append({"delta_parameters": ts})
        nnz = int(np.count_nonzero(x[kept]))
        assert c.compressors[1].last_need_to_send_advance == 1 + nnz * (1.0 + math.ceil(math.log2(10))) / 32.0
        assert c.compressors[0].last_need_to_send_advance == K
    s.update()
    cfg = ROUND_OPTS["adam"]
    theta0 = _flat(theta)
    agg_ref.fedopt_update(theta, delta, v, msgs, "adam", cfg["lr"], cfg["betas"], cfg["tau"])
    assert gc.same_bits(_flat(s.delta_parameters), _flat(delta))
    exp_v, got_v = _flat(v), _flat(s.v_parameters)  # (adaptive tail tolerance: see _check_adaptive_tail)
    ulp_v = np.abs(exp_v.view(np.int32).astype(np.int64) - got_v.view(np.int32).astype(np.int64))
    assert ulp_v.max() <= 1 and (ulp_v > 0).mean() < 0.01
    exp_t, got_t = _flat(theta), _flat(list(s.model.parameters()))
    err = np.abs(exp_t.astype(np.float64) - got_t.astype(np.float64))
    assert np.all(err <= 1e-6 * np.abs(exp_t.astype(np.float64) - theta0) + np.spacing(np.abs(exp_t)))


def test_fold_records_rejects_bad_arguments():
    from fl_sim_amd import _lib, codec

    n, k = 5000, 50
    stride, _ = codec.stacked_wire_layout(n, k)
    rec = torch.zeros(stride, dtype=torch.uint8, device="cuda")
    d = torch.zeros(n, device="cuda")
    import ctypes

    P = ctypes.c_void_p
    with pytest.raises(_lib.FlcError, match="hold"):  # tensor sizes do not add up to n
        _lib.call("flc_fedopt_fold_records", (P * 1)(rec.data_ptr()), (ctypes.c_float * 1)(1.0), 1, n, k, 127,
                  (P * 1)(d.data_ptr()), None, None, (ctypes.c_int64 * 1)(n - 1), 1, 0.0, 0, 1.0, 0.0, 0.0, None)
    with pytest.raises(_lib.FlcError, match="aligned"):
        _lib.call("flc_fedopt_fold_records", (P * 1)(rec.data_ptr() + 4), (ctypes.c_float * 1)(1.0), 1, n, k, 127,
                  (P * 1)(d.data_ptr()), None, None, (ctypes.c_int64 * 1)(n), 1, 0.0, 0, 1.0, 0.0, 0.0, None)
    with pytest.raises(_lib.FlcError, match="v required"):
        _lib.call("flc_fedopt_fold_records", (P * 1)(rec.data_ptr()), (ctypes.c_float * 1)(1.0), 1, n, k, 127,
                  (P * 1)(d.data_ptr()), (P * 1)(d.data_ptr()), None, (ctypes.c_int64 * 1)(n), 1, 0.0, 3, 1.0, 0.0,
                  0.0, None)


def test_stacked_message_fast_path_equals_the_converted_path():
    """Philox mode: the one-C-call message (_flcfold.stacked_delta_record on the parameters as they are) and the
    converted path (a client whose parameters live on the host, or are non-contiguous / float64: the tensors copied to
    contiguous fp32 device tensors first) give the same record, the same send statistics and the same Philox stream."""
    from fl_sim_amd import codec
    from fl_sim_amd.compressed import compress_delta

    assert codec._pydelta() is not None, "the _flcfold extension must be built"
    g = torch.Generator().manual_seed(11)
    shapes = [(16, 1, 5, 5), (16,), (256, 37), (10,)]
    glob = [torch.randn(sh, generator=g) for sh in shapes]
    loc = [t + torch.randn(t.shape, generator=g) * 1e-2 for t in glob]
    D = sum(t.numel() for t in glob)
    forms = {
        "device": ([t.cuda() for t in loc], [t.cuda() for t in glob]),
        "host": (loc, [t.cuda() for t in glob]),
        "noncontig": ([t.cuda() if i != 2 else t.cuda().t().contiguous().t() for i, t in enumerate(loc)],
                      [t.cuda() for t in glob]),
        "float64": ([t.double().cuda() for t in loc], [t.cuda() for t in glob]),
    }
    recs, stats = {}, {}
    for name, (ls, gs) in forms.items():
        comps = make_compressors("stacked10", D, rng="philox", seed=5)
        d = compress_delta(ls, gs, comps)
        pk = codec.wire_packet(d.record, D, d.k, d.levels)  # (the fields: a record's padding is never written)
        recs[name] = np.concatenate([pk.norm.cpu().numpy().view(np.uint8), pk.idx.cpu().numpy().view(np.uint8),
                                     pk.codes[:d.k].cpu().numpy(), pk.tiles.cpu().numpy().view(np.uint8)])
        stats[name] = (comps[0].total_input_components, comps[0].really_need_to_send_components,
                       comps[1].total_input_components, comps[1].really_need_to_send_components,
                       comps[1].last_need_to_send_advance, comps[1].philox.counter)
    assert not forms["noncontig"][0][2].is_contiguous()
    for name in ("host", "noncontig", "float64"):  # (the float64 copies of fp32 values convert back exactly)
        assert np.array_equal(recs[name], recs["device"]), name
        assert stats[name] == stats["device"], name


def test_pending_send_counts_written_on_side_streams_read_on_another():
    """Philox-mode messages made on side streams (their send counts left in the compressor's device slab) and the
    statistics read on the default stream: the read-back waits for the streams that wrote the counts, so the totals
    equal those of the same messages made on the default stream."""
    from fl_sim_amd.compressed import compress_delta

    g = torch.Generator().manual_seed(12)
    shapes = [(64, 3, 3), (4096,), (300, 77)]
    glob = [torch.randn(sh, generator=g).cuda() for sh in shapes]
    locs = [[t + torch.randn(t.shape, generator=g).cuda() * 1e-2 for t in glob] for _ in range(6)]
    D = sum(t.numel() for t in glob)

    def run(streams):
        comps = make_compressors("stacked10", D, rng="philox", seed=9)
        for i, ls in enumerate(locs):
            s = streams[i % len(streams)] if streams else None
            if s is None:
                compress_delta(ls, glob, comps)
            else:
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    big = torch.empty(1 << 26, device="cuda")  # (a long fill ahead of the count on that stream)
                    big.fill_(1.0)
                    compress_delta(ls, glob, comps)
        return (comps[1].total_input_components, comps[1].really_need_to_send_components,
                comps[1].last_need_to_send_advance)

    ref = run(None)
    got = run([torch.cuda.Stream(), torch.cuda.Stream()])
    assert got == ref


def _record_fields(d):
    from fl_sim_amd import codec

    pk = codec.wire_packet(d.record, d.n, d.k, d.levels)  # (the fields: a record's padding is never written)
    return np.concatenate([pk.norm.cpu().numpy().view(np.uint8), pk.idx.cpu().numpy().view(np.uint8),
                           pk.codes[:d.k].cpu().numpy(), pk.tiles.cpu().numpy().view(np.uint8)])


@pytest.mark.parametrize("n_msgs", [1, 7, 70])
def test_deferred_round_encode_equals_the_immediate_encodes(n_msgs, monkeypatch):
    """Deferred philox messages (each delta flattened when the message is made, the round's encodes in one batched
    launch on first access) against the one-C-call encode per message: the same records, the same send statistics
    and Philox streams — with every client's model changed in place right after its message was made (the snapshot),
    two counters in one round (two batches), a statistic read mid-round (the batches run), a resetStats, and 70
    messages (a batch runs itself at 64)."""
    from fl_sim_amd import compressed

    g = torch.Generator().manual_seed(13)
    shapes = [(16, 1, 5, 5), (16,), (256, 37), (10,)]
    glob = [torch.randn(sh, generator=g).cuda() for sh in shapes]
    D = sum(t.numel() for t in glob)
    locs = [[t + torch.randn(t.shape, generator=g).cuda() * 1e-2 for t in glob] for _ in range(n_msgs)]

    def run(defer):
        monkeypatch.setattr(compressed, "DEFER_ENCODE", defer)
        comps = [make_compressors("stacked10", D, rng="philox", seed=100 + i) for i in range(n_msgs)]
        for i in range(0, n_msgs, 3):  # (every third client's dithering stream one call ahead: a second counter)
            comps[i][1].philox.next()
        ls = [[t.clone() for t in loc] for loc in locs]
        ds, seen = [], []
        for i in range(n_msgs):
            ds.append(compressed.compress_delta(ls[i], glob, comps[i]))
            for t in ls[i]:
                t.add_(1.0)  # (the model moves on: the message keeps the delta it was made from)
            if i == n_msgs // 2:
                seen.append(comps[0][1].really_need_to_send_components)  # (a read mid-round)
            if i == 2:
                comps[1][1].resetStats()
        recs = [_record_fields(d) for d in ds]
        stats = [(c[0].total_input_components, c[1].total_input_components, c[1].really_need_to_send_components,
                  c[1].last_need_to_send_advance, c[1].philox.counter) for c in comps]
        return recs, stats, seen

    ra, sa, ma = run(True)
    assert not compressed._PENDING
    rb, sb, mb = run(False)
    for i, (x, y) in enumerate(zip(ra, rb)):
        assert np.array_equal(x, y), i
    assert sa == sb and ma == mb


def test_deferred_messages_of_many_counters_stay_bounded(monkeypatch):
    """Messages nobody reads, each of its own Philox counter (a batch each): past 16 waiting batches they are encoded,
    and every record and statistic still equals the immediate encodes'."""
    from fl_sim_amd import compressed

    g = torch.Generator().manual_seed(14)
    shapes = [(64, 9), (300,)]
    glob = [torch.randn(sh, generator=g).cuda() for sh in shapes]
    D = sum(t.numel() for t in glob)
    locs = [[t + torch.randn(t.shape, generator=g).cuda() * 1e-2 for t in glob] for _ in range(20)]

    def run(defer):
        monkeypatch.setattr(compressed, "DEFER_ENCODE", defer)
        comps = [make_compressors("stacked10", D, rng="philox", seed=7 + i) for i in range(20)]
        ds = []
        for i, c in enumerate(comps):
            for _ in range(i):
                c[1].philox.next()
            ds.append(compressed.compress_delta(locs[i], glob, c))
            if defer:
                assert len(compressed._PENDING) <= compressed._DEFER_MAX_BATCHES + 1
        return [_record_fields(d) for d in ds], [(c[1].really_need_to_send_components, c[1].philox.counter)
                                                  for c in comps]

    ra, sa = run(True)
    rb, sb = run(False)
    assert all(np.array_equal(x, y) for x, y in zip(ra, rb)) and sa == sb


def test_deferred_message_pickles_with_its_record():
    """A deferred message copied or pickled before anything read it carries the record its encode makes."""
    import copy
    import pickle

    from fl_sim_amd import compressed

    g = torch.Generator().manual_seed(15)
    glob = [torch.randn(4000, generator=g).cuda()]
    loc = [glob[0] + torch.randn(4000, generator=g).cuda() * 1e-2]
    comps = make_compressors("stacked10", 4000, rng="philox", seed=3)
    d = compressed.compress_delta(loc, glob, comps)
    assert d._batch is not None  # (deferred)
    c = copy.deepcopy(d)
    p = pickle.loads(pickle.dumps(d))
    ref = _record_fields(d)
    for x in (c, p):
        assert x._batch is None and np.array_equal(_record_fields(x), ref)
        assert torch.equal(torch.cat([t.reshape(-1) for t in x]).cpu(), torch.cat([t.reshape(-1) for t in d]).cpu())
