#!/bin/bash
# round 4: the headline decode's wave shape A/B on one box (FLC_LIB runs of the LIBS list, interleaved twice):
# tools/decode_probe.py (decode alone + the output's sha256, equal across libraries = bit-identical) and
# tools/calib_enc.py (encode / decode probes and the 1 GiB step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/${TAG:-decab}; mkdir -p $O
for rep in 1 2; do
  for kv in $LIBS; do
    echo "== ${kv%%=*}" >> $O/ab.txt
    FLC_LIB=${kv#*=} timeout -k 10 120 python -u tools/decode_probe.py >> $O/ab.txt 2>&1 || exit 1
    FLC_LIB=${kv#*=} SEED=1234 timeout -k 10 120 python -u tools/calib_enc.py 2>&1 | grep -E "decode|step" >> $O/ab.txt || exit 1
  done
done
grep -v amdgpu.ids $O/ab.txt
