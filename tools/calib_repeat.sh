#!/bin/bash
# Run-to-run variance of the per-kernel times: the same build, REPEAT fresh processes per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUTF=gpurun_out/calib_repeat.txt
: > $OUTF
for V in ${FILTER_VARIANTS:-0}; do
  [ "$V" != 0 ] && { make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_f$V.so BUILD=/tmp/bf$V EXTRA=-DFLC_FILTER_VARIANT=$V > /dev/null || exit 1; }
done
for r in $(seq ${REPEAT:-3}); do
  for V in ${FILTER_VARIANTS:-0}; do
    LIB=fl_sim_amd/libflcodec.so; [ "$V" != 0 ] && LIB=/tmp/libflc_f$V.so
    FLC_LIB=$LIB timeout -k 10 120 python tools/calib_filter.py "rep$r filter_v$V" >> $OUTF 2>&1
    rc=$?; [ $rc -ne 0 ] && { cat $OUTF; exit $rc; }
  done
done
grep -v amdgpu.ids $OUTF
