#!/bin/bash
# Calibration builds with arbitrary EXTRA flags: CONFIGS="name1:flags1;name2:flags2" -> /tmp/libflc_<name>.so,
# each timed REPEAT times with tools/calib_filter.py.  Variant results are for timing only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUTF=gpurun_out/calib_build.txt
: > $OUTF
IFS=';' read -ra CFG <<< "${CONFIGS}"
for c in "${CFG[@]}"; do
  name=${c%%:*}; flags=${c#*:}
  make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_$name.so BUILD=/tmp/b_$name EXTRA="$flags" > /dev/null || exit 1
done
for r in $(seq ${REPEAT:-2}); do
  for c in "${CFG[@]}"; do
    name=${c%%:*}
    FLC_LIB=/tmp/libflc_$name.so timeout -k 10 120 python tools/calib_filter.py "rep$r $name" >> $OUTF 2>&1
    rc=$?; [ $rc -ne 0 ] && { cat $OUTF; exit $rc; }
  done
done
grep -v amdgpu.ids $OUTF
