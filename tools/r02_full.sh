# round-2 evidence pass: GPU tests + smoke, driver-shaped bench line, headline rocprof summary; TAG names outputs
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r02}
bash tools/r02_gpu_all.sh $TAG || exit $?
timeout -k 10 500 python -u bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit $?
tail -1 gpurun_out/${TAG}_bench.log
bash tools/profile.sh ${TAG}_headline --skip-extra --skip-cpu --steps 20
