#!/bin/bash
# round-3 evidence pass: targeted GPU tests (TESTS), the whole GPU suite + smoke, the driver-shaped bench line,
# the headline rocprof summary.  Every GPU step has its own limit; the first failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r03}
run() {  # run <name> <limit-s> <cmd...>
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/${TAG}_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
PT="python -u -m pytest -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
[ -n "${TESTS:-}" ] && run targeted 600 $PT $TESTS
[ -z "${SKIP_SUITE:-}" ] && run gpu_tests 900 $PT tests
[ -z "${SKIP_SUITE:-}" ] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python -u bench.py --steps 20 --warmup 5
tail -1 gpurun_out/${TAG}_bench.log > gpurun_out/${TAG}_bench_line.json
[ -z "${SKIP_PROF:-}" ] && bash tools/profile.sh ${TAG}_headline --skip-extra --skip-cpu --steps 20
exit 0
