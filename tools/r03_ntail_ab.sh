#!/bin/bash
# same-box A/B of the decode's non-temporal tail (FLC_DECODE_NT_TAIL per-mille of the output written with NT stores,
# so fewer of its dirty lines are left in the Infinity Cache when the next encode streams): the headline bench line
# (step time, encode / decode kernel times), interleaved over two rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03}_ntail_ab.txt
: > $OUT
for round in 1 2; do
  for pm in ${VALS:-0 150 250 400 1000}; do
    FLC_DECODE_NT_TAIL=$pm timeout -k 10 120 python -u bench.py --skip-extra --skip-cpu --steps 40 --warmup 10 \
      > gpurun_out/ntail.log 2>&1 || exit $?
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ntail.log').read().strip().splitlines()[-1])
print('round $round nt_tail_pm $pm', 'ms', d['ms_per_step'], 'GB_s', d['value'], 'kernels_us', d['extra'].get('kernels_us'))" | tee -a $OUT
  done
done
