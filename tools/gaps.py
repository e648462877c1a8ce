"""Gaps between consecutive kernels of the headline step from a rocprofv3 --kernel-trace CSV (the last 20 steps of
tools/calib_enc.py's step loop): per kernel its median duration and the median idle time before it.
    python tools/gaps.py <kernel_trace.csv>"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
short = lambda s: ("topk_sample" if "topk_sample" in s else "stacked_encode" if "topk_select_kernel" in s  # noqa: E731
                   else "stacked_decode" if "sparse_decode" in s else s[:40])
seq = [(short(n), a, b) for n, a, b in ks]
# the step loop's tail: sample, encode, decode triples
trip = []
for i in range(len(seq) - 2):
    if [s[0] for s in seq[i:i + 3]] == ["topk_sample", "stacked_encode", "stacked_decode"]:
        trip.append(i)
trip = trip[-20:]
stat = {}
for i in trip:
    for j in range(3):
        n, a, b = seq[i + j]
        prev_end = seq[i + j - 1][2]
        stat.setdefault(n, []).append(((b - a) / 1e3, (a - prev_end) / 1e3))
for n, v in stat.items():
    print(f"{n:16s} duration {statistics.median([d for d, _ in v]):7.1f} us   gap before {statistics.median([g for _, g in v]):5.1f} us")
steps = [(seq[trip[q + 1]][1] - seq[trip[q]][1]) / 1e3 for q in range(len(trip) - 1)]
print(f"step (sample start to next sample start) median {statistics.median(steps):.1f} us")
