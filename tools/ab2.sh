#!/bin/bash
# Same-box A/B of two prebuilt libraries (ab/libflc_A.so = the base, ab/libflc_B.so = the change; built on the CPU
# side, the box only runs them): tools/calib_enc.py's per-kernel and step times, interleaved A B A B A B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  for v in A B; do
    echo "== $v round $r"
    FLC_LIB=ab/libflc_$v.so SEED=1234 timeout -k 10 100 python tools/calib_enc.py 2>&1 | grep -E "fused us|decode us|step" || exit 1
  done
done
