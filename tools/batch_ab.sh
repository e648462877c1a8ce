#!/bin/bash
# round 4: the batched encodes' parity tests, then tools/batch_host_probe.py with each library of LIBS (FLC_LIB runs,
# interleaved twice): synced and host-enqueue time per 100 x 1 M call.
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-batchab}; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $O/tests.txt 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for rep in 1 2; do
  for kv in $LIBS; do
    echo "== ${kv%%=*}" >> $O/ab.txt
    FLC_LIB=${kv#*=} timeout -k 10 120 python -u tools/batch_host_probe.py 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || exit 1
  done
done
cat $O/ab.txt
