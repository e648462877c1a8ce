"""Phase stamps of the float64 top-k (diagnostic build: tools/build_diag.sh, FLC_LIB=diag/libflcodec_stamps.so).

Slots (s_memrealtime, 100 MHz), f64.hip STAMP64: 0 sample block 0 start, 1 floor start, 2 band found; 3 filter block 0 start, 4 filter block 0 end; 5 select block 0 start, 6 its band histogram published,
7 past barrier 1, 8 its bin slice summed, 9 past barrier 2, 10 the K-th largest's bin found, 11 its keys appended,
12 past barrier 3, 13 T resolved; 14 emit block 0 start.  Times in us relative to slot 0."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from fl_sim_amd import codec  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 25_000_000
k = n // 100
x = torch.randn(n, generator=torch.Generator(device="cuda").manual_seed(5), device="cuda", dtype=torch.float64)
nch = -(-n // 8192)
al = lambda v: -(-v // 256) * 256  # noqa: E731
off = al(nch * 4) + al((nch + 1) * 8) + al(nch * 8)  # carve64: counts, offsets, part, then Sel64
names = ["sample0", "floor", "band", "filt0", "filt0end", "sel0", "hist", "bar1", "slice", "bar2", "bin", "append",
         "bar3", "T", "emit0"]
rows = []
for it in range(12):
    codec.topk_dense_f64(x, k)
    torch.cuda.synchronize()
    ws = codec._WS[(0, codec._stream(x.device), "f64")]
    st = ws[off:off + 15 * 8].cpu().numpy().view(np.uint64).astype(np.int64)
    if it >= 2:
        rows.append((st - st[0]) / 100.0)
m = np.median(np.array(rows), axis=0)
print("median us since sample start:", " ".join(f"{nm}={v:.1f}" for nm, v in zip(names, m)))
for r in rows[:3]:
    print(" ".join(f"{v:.1f}" for v in r))
