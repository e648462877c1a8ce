"""Host-side logic of the codec's call site (fl_sim_amd/compressed.py), no GPU: which compressor sequences make the
stacked wire, the message's delta as a sequence of tensors, a round's records recognised for the fused fold, and
the ClientMessage stand-in (nodes.py:1537-1557)."""

import numpy as np
import torch

from fl_sim_amd import Compressor
from fl_sim_amd.compressed import ClientMessage, CompressedDelta, client_message_class, stacked_pipeline, stacked_round


def _std(L, p, fp64=False):
    c = Compressor()
    nc = Compressor("norm")
    nc.makeIdenticalCompressor()
    (c.makeStandardDitheringFP64 if fp64 else c.makeStandardDitheringFP32)(L, nc, p)
    return c


def _topk(K=10, D=1000):
    c = Compressor()
    c.makeTopKCompressor(K, D)
    return c


def test_stacked_pipeline_detection():
    assert stacked_pipeline([_topk(), _std(10, np.inf)]) == (10, 10)
    assert stacked_pipeline([_topk(7), Compressor(extended_levels=True)]) is None  # (an identical compressor)
    big = Compressor(extended_levels=True)
    nc = Compressor("norm")
    nc.makeIdenticalCompressor()
    big.makeStandardDitheringFP32(127, nc, np.inf)
    assert stacked_pipeline([_topk(7), big]) == (7, 127)
    assert stacked_pipeline([_topk(), _std(8, 2)]) is None          # p = 2: not the wire's p = inf
    assert stacked_pipeline([_topk(), _std(8, np.inf, True)]) is None  # float64 stage
    assert stacked_pipeline([_std(8, np.inf), _topk()]) is None     # order matters
    assert stacked_pipeline([_topk()]) is None


def test_compressed_delta_is_a_sequence_of_the_model_tensors():
    flat = torch.arange(2 * 3 + 4 + 1, dtype=torch.float32)
    d = CompressedDelta([(2, 3), (4,), (1,)], torch.device("cpu"), flat.numel(), flat=flat)
    assert d.kind == "dense" and len(d) == 3 and d.nbytes == 4 * 11
    ts = list(d)
    assert [tuple(t.shape) for t in ts] == [(2, 3), (4,), (1,)]
    assert torch.equal(torch.cat([t.reshape(-1) for t in ts]), flat)
    assert torch.equal(d[1], flat[6:10])


def test_stacked_round_recognises_one_shape_of_records():
    rec = torch.zeros(256, dtype=torch.uint8)
    a = CompressedDelta([(100,)], torch.device("cpu"), 100, record=rec, k=1, levels=10)
    b = CompressedDelta([(100,)], torch.device("cpu"), 100, record=rec, k=1, levels=10)
    c = CompressedDelta([(100,)], torch.device("cpu"), 100, record=rec, k=2, levels=10)
    dense = CompressedDelta([(100,)], torch.device("cpu"), 100, flat=torch.zeros(100))
    assert stacked_round([{"delta_parameters": a}, {"delta_parameters": b}]) == [a, b]
    assert stacked_round([{"delta_parameters": a}, {"delta_parameters": c}]) is None
    assert stacked_round([{"delta_parameters": a}, {"delta_parameters": dense}]) is None
    assert stacked_round([{"delta_parameters": [torch.zeros(3)]}]) is None
    assert stacked_round([]) is None


def test_client_message_stand_in():
    cls = client_message_class()
    m = cls(client_id=3, train_samples=17, metrics={}, delta_parameters=[])
    assert isinstance(m, dict) and m["client_id"] == 3 and m["train_samples"] == 17
    assert ClientMessage(1, 2, {}, x=5)["x"] == 5


def test_pending_send_statistics_fold_in_on_read():
    """A philox-mode compressed round leaves the dithering stage's count on the device; reading a counter folds it in
    with the reference's arithmetic (compressors.py:362-365, 406-408)."""
    c = _std(10, np.inf)
    c._finish(50, 3.0)
    c._finish_pending(100, torch.tensor([7]), 1, 5.0 / 32.0)
    assert c.total_input_components == 150
    assert c.last_need_to_send_advance == 1 + 7 * 5.0 / 32.0
    assert c.really_need_to_send_components == 3.0 + 1 + 7 * 5.0 / 32.0
    c._finish_pending(100, torch.tensor([0]), 1, 5.0 / 32.0)
    c.resetStats()
    assert c.really_need_to_send_components == 0 and c.last_need_to_send_advance == 0


def test_pending_send_statistics_of_many_calls_fold_in_call_order():
    """Counts of several philox-mode calls wait together (read back in one copy, at most 64 at a time) and fold in
    call by call: the totals and the last call's advance equal those of the calls finished one at a time."""
    per = 5.0 / 32.0
    counts = [7, 0, 3, 11, 0, 2] + list(range(70))
    a, b = _std(10, np.inf), _std(10, np.inf)
    for cnt in counts:
        a._finish_pending(100, torch.tensor([cnt]), 1, per)
        b._finish(100, 1 + cnt * per if cnt else 1)
    assert len(a.__dict__.get("_pending") or []) <= 64
    assert a.total_input_components == b.total_input_components
    assert a.really_need_to_send_components == b.really_need_to_send_components
    assert a.last_need_to_send_advance == b.last_need_to_send_advance


def test_pending_counts_in_slab_slots_fold_in_call_order():
    """The counts written into the compressor's slab slots (_count_slot, as compressed.py's philox path writes them)
    fold in exactly as counts finished one at a time, across slab refills; a slot handed out but never finished (a
    call that fell through to another path) is handed out again."""
    per = 5.0 / 32.0
    cpu = torch.device("cpu")
    counts = [7, 0, 3] + list(range(140))
    a, b = _std(10, np.inf), _std(10, np.inf)
    for i, cnt in enumerate(counts):
        slot = a._count_slot(cpu)
        if i == 5:
            assert a._count_slot(cpu).data_ptr() == slot.data_ptr()  # (unfinished: the same slot again)
        slot.fill_(cnt)
        a._finish_pending(100, slot, 1, per)
        b._finish(100, 1 + cnt * per if cnt else 1)
        if i == 70:
            assert a.last_need_to_send_advance == b.last_need_to_send_advance  # a read mid-slab frees the slots
    assert len(a.__dict__.get("_pending") or []) <= 64
    assert a.total_input_components == b.total_input_components
    assert a.really_need_to_send_components == b.really_need_to_send_components
    assert a.last_need_to_send_advance == b.last_need_to_send_advance


def test_copies_and_pickles_carry_the_pending_send_statistics():
    """A compressor with send counts still pending in its slab: a deep copy and a pickle round trip hold the folded
    statistics (and no slab); the original keeps working."""
    import copy
    import pickle

    per = 5.0 / 32.0
    cpu = torch.device("cpu")
    a, b = _std(10, np.inf), _std(10, np.inf)
    for cnt in (4, 0, 9):
        slot = a._count_slot(cpu)
        slot.fill_(cnt)
        a._finish_pending(100, slot, 1, per)
        b._finish(100, 1 + cnt * per if cnt else 1)
    for c in (copy.deepcopy(a), pickle.loads(pickle.dumps(a))):
        assert "_slab" not in c.__dict__ and not c.__dict__.get("_pending")
        assert c.really_need_to_send_components == b.really_need_to_send_components
        assert c.last_need_to_send_advance == b.last_need_to_send_advance
        assert c.total_input_components == b.total_input_components
    slot = a._count_slot(cpu)
    slot.fill_(2)
    a._finish_pending(100, slot, 1, per)
    b._finish(100, 1 + 2 * per)
    assert a.really_need_to_send_components == b.really_need_to_send_components
