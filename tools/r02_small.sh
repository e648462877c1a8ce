set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r02g}
timeout -k 10 120 python tools/small_configs.py > gpurun_out/${TAG}_small.log 2>&1 || exit $?
cat gpurun_out/${TAG}_small.log | grep us/step
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/${TAG}_small -o run --output-format csv -- python3 tools/small_configs.py > gpurun_out/prof_${TAG}_small.log 2>&1 || exit $?
f=$(find gpurun_out/prof/${TAG}_small -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${TAG}_small_kernel_stats.csv
cut -d, -f1-4 gpurun_out/${TAG}_small_kernel_stats.csv | cut -c1-160
