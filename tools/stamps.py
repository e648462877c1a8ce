"""Phase stamps of the persistent encode (diagnostic build: make EXTRA=-DFLC_SELECT_STAMPS, block 0 only).

Stamp slots (s_memrealtime, 100 MHz): 0 start, 1 sample keys histogrammed, 2 floor/ceiling, 3 HBM pass done, 4 histogram flushed
(split path: staged); 5 select start (fused default: after the exchange that follows the filter phase),
6 loads done, 7 pick, 8 in-bin lists published, 9 exchanged, 10 list gathered, 11 T resolved, 12 sums,
13 counts, 14 keep decisions staged (x-mode: compaction done), 15 written out with the tile pointers.  FLC_TOPK_SPLIT=1 times the two-kernel path instead.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from fl_sim_amd import codec

STAMP_OFF = 234752  # byte offset of EncWs.stamps in the top-k workspace (topk.hip: kOffStamps, 8 histogram copies)
BLKT_OFF = 235008   # kOffBlkT
n = int(sys.argv[1]) if len(sys.argv) > 1 else 268_435_456
k = n // 100
seed = int(os.environ.get("SEED", "1"))  # bench.py's headline delta: SEED=1234
x = torch.randn(n, device="cuda", generator=torch.Generator(device="cuda").manual_seed(seed)) * 1e-3
if os.environ.get("DELTA"):  # f1: the delta-fused encode over 64 tensors (local = x piece + global, global random)
    gen = torch.Generator(device="cuda").manual_seed(seed + 1)
    sizes = [n // 64] * 63 + [n - 63 * (n // 64)]
    glo = [torch.randn(s, device="cuda", generator=gen) for s in sizes]
    loc = [gl + xp for gl, xp in zip(glo, torch.split(x, sizes))]
    encode = lambda it: codec.stacked_encode_delta(loc, glo, k, 127, seed=1, counter=it)
elif os.environ.get("BATCH"):  # the batched encode of 100 clients x 1 M: client 0's header (block 0 of client 0)
    gen = torch.Generator(device="cuda").manual_seed(seed + 2)
    xs = [torch.randn(1_000_000, device="cuda", generator=gen) * 1e-3 for _ in range(int(os.environ["BATCH"]))]
    encode = lambda it: codec.stacked_encode_batch(xs, 10_000, 127, seeds=list(range(len(xs))), counter=it)  # noqa: E731
elif os.environ.get("PLAIN"):  # the plain top-k select (configs[2]'s TopK compressor path)
    encode = lambda it: codec.topk_encode(x, k, with_tiles=True)  # noqa: E731
else:
    encode = lambda it: codec.stacked_encode(x, k, 127, 1, it)
names = ["keys", "sample-sel", "filter", "post+stage+flush", "boundary", "load", "pick0", "inbin", "x1", "list", "local", "sums", "counts", "decide", "write+tiles"]
for it in range(int(os.environ.get("ITERS", "12"))):
    encode(it)
    torch.cuda.synchronize()
    ws = [t for key, t in codec._WS.items() if key[2] == ("topk_batch" if os.environ.get("BATCH") else "topk")][0]
    st = ws[STAMP_OFF:STAMP_OFF + 16 * 8].cpu().numpy().view(np.uint64).astype(np.int64)
    if it < 2:
        continue
    sv = ws[:16 * 8].cpu().numpy().view(np.uint64)
    print("state call,err,C,fb,T,maxkey,rounds,t_lo,t_hi,need,ties,strict,path:", [int(v) for v in sv[:13]])
    t = st[:16].astype(np.float64)
    prev, parts = t[0], []
    for i in range(1, 16):
        if t[i] > 0 and t[i] >= prev:
            parts.append(f"{names[i - 1]} {(t[i] - prev) * 10 / 1000:.1f}")
            prev = t[i]
    print(" | ".join(parts), f"| total {(max(t[14], t[15]) - t[0]) * 10 / 1000:.1f} us")
    wrow = ws[BLKT_OFF + 768 * 32:BLKT_OFF + 800 * 32].cpu().numpy().view(np.uint64).astype(np.int64).reshape(32, 4)[:, 0]
    if wrow[16] > 0 and t[8] > 0:  # the speculative compaction's per-wave stamps (block 0), from stamp 8 (lists published)
        rel = lambda v: round(float(v - t[8]) * 10 / 1000, 1) if v > 0 else None  # noqa: E731
        print("  spec: workers start", rel(wrow[16]), "end per wave", [rel(v) for v in wrow[1:16]],
              "| wave 0: meta", rel(wrow[17]), "keys", rel(wrow[19]), "T", rel(wrow[20]), "counts", rel(wrow[21]))
        ws[BLKT_OFF + 768 * 32:BLKT_OFF + 800 * 32].zero_()
    ws[STAMP_OFF:STAMP_OFF + 16 * 8].zero_()
    if os.environ.get("XCD_EVERY"):  # per-call mean pass duration per XCD (blockIdx % 8), and the max block
        bt = ws[BLKT_OFF:BLKT_OFF + 256 * 32].cpu().numpy().view(np.uint64).astype(np.int64).reshape(256, 4)
        G = int((bt[:, 0] > 0).sum())
        d = (bt[:G, 1] - bt[:G, 0]) * 10 / 1000
        print("xcd means", [round(float(d[np.arange(G) % 8 == i].mean()), 1) for i in range(8)],
              "median", round(float(np.median(d)), 1), "max", round(float(d.max()), 1), "argmax", int(d.argmax()))
    if it == int(os.environ.get("ITERS", "12")) - 1:  # per-block filter times (start of the HBM pass, its end, end of the kernel)
        bt = ws[BLKT_OFF:BLKT_OFF + 256 * 32].cpu().numpy().view(np.uint64).astype(np.int64).reshape(256, 4)
        G = int((bt[:, 0] > 0).sum())
        bt = bt[:G]
        t0 = bt[:, 0].min()
        st_ = (bt[:, 0] - t0) * 10 / 1000
        en_ = (bt[:, 1] - t0) * 10 / 1000
        dur = en_ - st_
        print(f"blocks {G}: pass start spread {st_.max():.1f} us; pass duration min {dur.min():.1f} median {np.median(dur):.1f} max {dur.max():.1f}; last end {en_.max():.1f}")
        order = np.argsort(dur)
        print("slowest blocks:", [(int(b), round(float(dur[b]), 1)) for b in order[-8:]])
        xcd = np.arange(G) % 8
        print("mean duration by blockIdx % 8:", [round(float(dur[xcd == i].mean()), 1) for i in range(8)])
        cov = bt[:, 2]
        done, tot = (cov & 0xffffffff).astype(np.float64), (cov >> 32).astype(np.float64)
        frac = done / np.maximum(tot, 1)
        print(f"philox chunks precomputed: min {frac.min():.2f} median {np.median(frac):.2f} (of {int(np.median(tot))} per block)")
        if (bt[:, 3] > 0).all():  # kernel end per block (select / fused kernel)
            fin = (bt[:, 3] - t0) * 10 / 1000
            o = np.argsort(fin)
            print(f"kernel end: block 0 {fin[0]:.1f} us, min {fin.min():.1f}, median {np.median(fin):.1f}, "
                  f"max {fin.max():.1f}; last blocks:", [(int(b), round(float(fin[b]), 1)) for b in o[-6:]])
