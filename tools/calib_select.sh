#!/bin/bash
# Select-kernel ablations (calibration builds in /tmp, results invalid): compaction without Philox,
# without the output writes; phase stamps of each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "base:-DFLC_SELECT_STAMPS" "nophilox:-DFLC_SELECT_STAMPS -DFLC_CALIB_NOPHILOX=1" "nowrite:-DFLC_SELECT_STAMPS -DFLC_CALIB_NOWRITE=1"; do
  name=${v%%:*}; flags=${v#*:}
  make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_$name.so BUILD=/tmp/b_$name EXTRA="$flags" > /dev/null || exit 1
  echo "== $name"
  FLC_LIB=/tmp/libflc_$name.so timeout -k 10 120 python tools/stamps.py 2>&1 | grep compact | tail -2
done
