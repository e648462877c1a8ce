#!/bin/bash
# round 4: the batched 100 x 1 M stacked encode — synced vs host-enqueue time per call, then a rocprof kernel trace
# of the same probe: per-kernel averages and the last call's timeline (kernel start / end, us from its first kernel).
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-batchprof}; mkdir -p $O
timeout -k 10 120 python -u tools/batch_host_probe.py > $O/host.txt 2>&1 || exit 1
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/tools/batch_host_probe.py > $R/$O/prof.log 2>&1 || exit 1
cd $R; grep -v amdgpu.ids $O/host.txt
python3 - "$O" <<'PY'
import csv, glob, sys
o = sys.argv[1]
for r in csv.DictReader(open(glob.glob(f"{o}/prof/**/*kernel_stats.csv", recursive=True)[0])):
    print(r["Name"][:80], r["Calls"], r["AverageNs"])
rows = sorted(csv.DictReader(open(glob.glob(f"{o}/prof/**/*kernel_trace.csv", recursive=True)[0])),
              key=lambda r: int(r["Start_Timestamp"]))
last = rows[-12:]
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    print(r["Kernel_Name"][:60], (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3)
PY
