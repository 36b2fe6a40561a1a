#!/bin/bash
# Interleaved A/B of the C2 timed loop (tools/gs_c2.py), one process per arm, GS_AB_ROUNDS rounds:
#   tools/gs_ab.sh "<arm A env/args>" "<arm B env/args>" ...   e.g. tools/gs_ab.sh "" "PTGS_GS_HELPERS=always"
# An arm is "VAR=value ..." (GS_LIB=libptgs_<variant>.so picks a library); stops at the first failure.
set -euo pipefail
for i in $(seq 1 "${GS_AB_ROUNDS:-3}"); do
  for arm in "$@"; do
    env GS_TAG="${arm:-base}" $arm timeout -k 10 90 python3 tools/gs_c2.py
  done
done
