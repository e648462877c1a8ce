"""Phase stamps of the float64 top-k (diagnostic build: tools/build_diag.sh, FLC_LIB=diag/libflcodec_stamps.so).

Slots (s_memrealtime, 100 MHz), f64.hip STAMP64: 0 prep block 0 start; 5 select block 0 start, 6 band found,
7 its chunks filtered (histogram flushed), 8 past the barrier, 10 the K-th largest's bin found, 11 its keys appended,
12 every block's appends in, 15 the bin's list loaded, 13 T resolved; 14 emit block 0 start; inside the band: 16 the sample's keys in, 17 their
histogram, 18 the floor and ceiling bins picked (6: refined).  Per block (round 4):
the filter pass done and the histogram flushed (min / median / max over the blocks).  Times in us relative to
slot 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
k = n // 100
x = torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda", dtype=torch.float64)
# ROTATE=3: three distinct inputs in rotation (not cache-resident)
xs = [x] + [torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(6 + i), device="cuda",
                        dtype=torch.float64) for i in range(int(os.environ.get("ROTATE", "1")) - 1)]
nch = -(-n // 8192)
al = lambda v: -(-v // 256) * 256  # noqa: E731
off = al(32 * 8) + al(nch * 4) + al((nch + 1) * 8) + al(nch * 8)  # carve64: sticky word, counts, offsets, part, then Sel64
names = ["prep0", "", "", "", "", "sel0", "band", "filtered", "bar1", "", "bin", "append", "bar2", "T", "emit0",
         "list", "keys", "shist", "spick"]
G = torch.cuda.get_device_properties(0).multi_processor_count
rows, blk = [], []
for it in range(12):
    codec.topk_dense_f64(xs[it % len(xs)], k)
    torch.cuda.synchronize()
    ws = codec._WS[(0, codec._stream(x.device), "f64")]
    st = ws[off:off + 19 * 8].cpu().numpy().view(np.uint64).astype(np.int64)
    bs = ws[off + 256:off + 256 + 2 * 1024 * 8].cpu().numpy().view(np.uint64).astype(np.int64).reshape(2, 1024)
    if it >= 2:
        rows.append((st - st[0]) / 100.0)
        blk.append((bs[:, :G] - st[0]) / 100.0)
m = np.median(np.array(rows), axis=0)
print("median us since prep start:", " ".join(f"{nm}={v:.1f}" for nm, v in zip(names, m) if nm))
for r in rows[:3]:
    print(" ".join(f"{v:.1f}" for nm, v in zip(names, r) if nm))
b = np.median(np.array(blk), axis=0)
for i, nm in enumerate(["filter done", "hist flushed"]):
    print(f"per block {nm}: min {b[i].min():.1f} median {np.median(b[i]):.1f} max {b[i].max():.1f} "
          f"(block 0 {b[i][0]:.1f}; slowest blocks {np.argsort(b[i])[-4:].tolist()})")
