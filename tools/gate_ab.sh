#!/bin/bash
# same-box A/B of the co-residency gate (tools/gate_probe.py) between prebuilt libraries, interleaved A B A B ...
#   bash tools/gate_ab.sh OUTFILE lib1.so lib2.so [rounds]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; a=$2; b=$3; r=${4:-3}
for i in $(seq $r); do
  for lib in $a $b; do
    FLC_LIB=$lib timeout -k 10 120 python3 tools/gate_probe.py >> $out 2>&1 || exit 1
  done
done
cat $out
