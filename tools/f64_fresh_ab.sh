#!/bin/bash
# round 4: the float64 top-k per library of LIBS (FLC_LIB runs, interleaved twice), same input and three rotated inputs
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-f64fresh}; mkdir -p $O
for rep in 1 2; do
  for kv in $LIBS; do
    echo "== ${kv%%=*}" >> $O/ab.txt
    FLC_LIB=${kv#*=} timeout -k 10 120 python -u tools/topk64_probe.py 2>&1 | grep -E "matches|us/call" >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
