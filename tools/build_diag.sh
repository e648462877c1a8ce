#!/bin/bash
# Diagnostic build of libflcodec.so with the encode's phase stamps (tools/stamps.py: FLC_LIB=diag/libflcodec_stamps.so)
cd "$(dirname "$0")/.." && mkdir -p diag && make -C fl_sim_amd/csrc EXTRA=-DFLC_SELECT_STAMPS OUT=../../diag/libflcodec_stamps.so \
  BUILD=../../diag/obj ../../diag/libflcodec_stamps.so -j8
