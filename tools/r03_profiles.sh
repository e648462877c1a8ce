#!/bin/bash
# round 3: rocprofv3 kernel-trace summaries of the small configs, adaptive random (25 M) and the aggregation kernels.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r03}
for P in small_configs adaptive_probe agg_probe; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_$P -o run --output-format csv \
    -- python3 tools/$P.py > gpurun_out/${TAG}_$P.log 2>&1 || exit $?
  grep -E "us/|ms per" gpurun_out/${TAG}_$P.log
  f=$(find gpurun_out/prof/${TAG}_$P -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${TAG}_${P}_kernel_stats.csv
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_${P}_kernel_stats.csv')):
    print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3, 2), 'us')" | head -14
done
