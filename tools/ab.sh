#!/bin/bash
# A/B timing on ONE box: library A = HEAD's sources (git stash-free: built from a worktree copy), B = the
# working tree.  Each is timed twice, interleaved (box-to-box variance is ~10 %, in-box ~1 %).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=${A_DIR:-/tmp/ab_a}
make -s -C $A/fl_sim_amd/csrc -j16 OUT=/tmp/libflc_A.so BUILD=/tmp/b_A > /dev/null || exit 1
make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_B.so BUILD=/tmp/b_B > /dev/null || exit 1
for r in 1 2; do
  for v in A B; do
    echo "== $v"; FLC_LIB=/tmp/libflc_$v.so SEED=1234 timeout -k 10 100 python tools/calib_enc.py 2>&1 | grep -E "filter us|decode|step"
  done
done
