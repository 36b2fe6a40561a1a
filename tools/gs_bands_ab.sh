#!/bin/bash
# Band frame times (tools/gs_bands.py, no profiler) of two libraries, interleaved: C2 and 10M at 4K,
# the full frame and bands 0 / 3 of 8 with chunk bounds. GS_LIBS="libptgs.so libptgs_cullk.so"
set -euo pipefail
for cfg in ${GS_CFGS:-c2 10m}; do
  for band in full 0 3; do
    for lib in ${GS_LIBS:-libptgs.so libptgs_cullk.so}; do
      GS_LIB=$lib GS_CFG=$cfg GS_BAND=$band GS_BOUNDS=1 timeout -k 10 200 python3 tools/gs_bands.py
    done
  done
done
