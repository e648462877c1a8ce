#!/bin/bash
# Same-box A/B of two prebuilt libraries on the aggregation kernels (tools/agg_probe.py: wall time per call, then a
# rocprofv3 kernel-trace summary per library):  LIBS="A=ab/libflc_A.so B=ab/libflc_B.so" bash tools/agg_ab.sh
# Each library is copied over the in-tree fl_sim_amd/libflcodec.so of the box's copy of the tree (the _flcfold
# extension links that file, whatever FLC_LIB says).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && export TMPDIR=/tmp && mkdir -p gpurun_out/aggab
for rep in 1 2; do
  for kv in $LIBS; do
    echo "== ${kv%%=*}"
    cp ${kv#*=} fl_sim_amd/libflcodec.so && timeout -k 10 120 python -u tools/agg_probe.py 2>&1 | grep us/call || exit 1
  done
done
for kv in $LIBS; do
  cp ${kv#*=} fl_sim_amd/libflcodec.so && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/aggab/${kv%%=*} -o run \
    --output-format csv -- python3 tools/agg_probe.py > /dev/null 2>&1 || exit 1
  f=$(find gpurun_out/aggab/${kv%%=*} -name "*kernel_stats.csv" | head -1)
  echo "== ${kv%%=*} kernels"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')"
done
