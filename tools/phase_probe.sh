#!/bin/bash
# Encode-phase stamps (diagnostic build in /tmp) + kernel timeline of the headline step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
make -s -C fl_sim_amd/csrc -j16 OUT=/tmp/libflc_stamps.so BUILD=/tmp/b_stamps EXTRA="-DFLC_SELECT_STAMPS" > /dev/null || exit 1
FLC_LIB=/tmp/libflc_stamps.so timeout -k 10 120 python tools/stamps.py "$@" > gpurun_out/stamps.txt 2>&1 || { cat gpurun_out/stamps.txt; exit 1; }
cat gpurun_out/stamps.txt
