set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r02a_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r02a_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r02a_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r02a_bench.log
bash tools/profile.sh r02a_headline --skip-extra --skip-cpu --steps 20
