#!/bin/bash
# round 4: the float64 top-k A/B on one box, FLC_LIB runs (diag/lib_base.so = the library before the change).
# Parity tests first, then each library of LIBS timed twice (interleaved), the phase stamps of each STAMPS library and
# a rocprof kernel summary of the in-tree library.
#   TAG=r04x LIBS="base=diag/lib_base.so new=fl_sim_amd/libflcodec.so" STAMPS="new=diag/libflcodec_stamps.so" \
#     bash tools/f64_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-f64ab}; mkdir -p $O
LIBS=${LIBS:-"base=diag/lib_base.so new=fl_sim_amd/libflcodec.so"}
STAMPS=${STAMPS:-"new=diag/libflcodec_stamps.so"}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_f64.py > $O/tests_f64.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/tests_f64.txt; exit 1; }
tail -2 $O/tests_f64.txt
for rep in 1 2; do
  for kv in $LIBS; do
    echo "== ${kv%%=*}" >> $O/probe.txt
    FLC_LIB=${kv#*=} timeout -k 10 120 python -u tools/topk64_probe.py >> $O/probe.txt 2>&1 || exit 1
  done
done
for kv in $STAMPS; do
  echo "== ${kv%%=*}" >> $O/stamps.txt
  FLC_LIB=${kv#*=} timeout -k 10 120 python -u tools/stamps64.py >> $O/stamps.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/topk64_probe.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT; grep -E '^==|us/call|matches' $O/probe.txt; grep -v amdgpu.ids $O/stamps.txt
