#!/bin/bash
# HBM traffic of the headline kernels from rocprofv3 PMC counters, one counter per pass (FETCH_SIZE and
# WRITE_SIZE do not fit one TCC pass on gfx950), then tools/traffic.py -> gpurun_out/traffic.json.
# Counters run with --kernel-trace only (no sys/runtime traces).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
TAG=${1:-pmc}
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc/${TAG}_$C -o run --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --skip-extra --skip-cpu > gpurun_out/pmc/${TAG}_$C.log 2>&1
  rc=$?
  echo "pmc $C rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
python3 tools/traffic.py gpurun_out/pmc $TAG > gpurun_out/traffic.json && cat gpurun_out/traffic.json
