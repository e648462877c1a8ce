#!/bin/bash
# round-6 GPU pass: targeted tests (TESTS=...), the driver-shaped bench line, the headline-only rocprof summary.
# Each GPU step under its own time limit, chained so that nothing runs after a failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r06x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rc=0
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_LIMIT:-600} python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu $TESTS \
    > $OUT/tests.log 2>&1; rc=$?
  tail -3 $OUT/tests.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  timeout -k 10 420 python3 bench.py --steps 20 --warmup 5 > $OUT/bench_line.json 2> $OUT/bench.err; rc=$?
  tail -c 400 $OUT/bench_line.json
  [ $rc -ne 0 ] && exit $rc
fi
if [ -z "${SKIP_PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --skip-extra --skip-cpu > $OUT/prof.log 2>&1; rc=$?
  find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/headline_kernel_stats.csv \;
  head -5 $OUT/headline_kernel_stats.csv | cut -c1-160
fi
exit $rc
