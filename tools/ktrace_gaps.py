"""Per kernel name (shortened): median duration and median idle time before it, over the last `last` kernels of a
rocprofv3 --kernel-trace CSV.   python tools/ktrace_gaps.py <kernel_trace.csv> [last]"""
import csv
import statistics
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 60
ks = [(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
ks = ks[-last - 1:]
stat = {}
for (n0, a0, b0), (n, a, b) in zip(ks, ks[1:]):
    stat.setdefault(n, []).append(((b - a) / 1e3, (a - b0) / 1e3))
for n, v in stat.items():
    print(f"{n:60s} x{len(v):3d} duration {statistics.median([d for d, _ in v]):7.1f} us"
          f"   gap before {statistics.median([g for _, g in v]):6.1f} us")
