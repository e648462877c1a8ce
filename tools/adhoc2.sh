#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for V in "" "-DFLC_CALIB_NOPHILOX=1" "-DFLC_CALIB_NOWRITE=1"; do
  make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_st.so BUILD=/tmp/b_st EXTRA="-DFLC_SELECT_STAMPS $V" > /dev/null || exit 1
  echo "== $V"; ITERS=5 SEED=1234 FLC_LIB=/tmp/libflc_st.so timeout -k 10 120 python tools/stamps.py 2>&1 | grep -v amdgpu.ids | grep -v state | grep -E "compact|philox|kernel end"
  rm -rf /tmp/b_st
done
