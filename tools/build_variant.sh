#!/bin/bash
# build_variant.sh NAME "EXTRA FLAGS": diag/lib_NAME.so (libflcodec.so with extra -D flags, e.g. the encode's phase
# stamps -DFLC_SELECT_STAMPS or calibration switches), for FLC_LIB=diag/lib_NAME.so runs of tools/stamps.py / calib_enc.py
cd "$(dirname "$0")/.." && mkdir -p diag && make -s -C fl_sim_amd/csrc EXTRA="$2" OUT=../../diag/lib_$1.so \
  BUILD=../../diag/obj_$1 ../../diag/lib_$1.so -j8
