#!/bin/bash
# Calibration builds of the filter / decode (results of variants != 0 are NOT valid top-k output):
# each variant is built into /tmp and timed with tools/calib_filter.py via FLC_LIB.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
OUTF=gpurun_out/calib_variants.txt
: > $OUTF
for V in ${FILTER_VARIANTS:-0 1 2}; do
  make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_f$V.so BUILD=/tmp/bf$V EXTRA=-DFLC_FILTER_VARIANT=$V > /dev/null || exit 1
done
for V in ${FILTER_VARIANTS:-0 1 2}; do
  for DV in ${DECODE_VARIANTS:-40 90}; do
    FLC_LIB=/tmp/libflc_f$V.so FLC_DECODE_VARIANT=$DV timeout -k 10 120 python tools/calib_filter.py "filter_v$V decode_v$DV" >> $OUTF 2>&1
    rc=$?
    [ $rc -ne 0 ] && { echo "rc=$rc"; cat $OUTF; exit $rc; }
  done
done
cat $OUTF
