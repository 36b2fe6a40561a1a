#!/bin/bash
# One parametrised gpurun step driver (replaces round 5's one-off tools/r05_check*.sh scripts):
#   tools/gpu_steps.sh <out-dir> "<seconds>|<name>|<command>" ...
# Each step runs under its own `timeout -k 10 <seconds>` from the repo root, with stdout + stderr in
# <out-dir>/<name>.log; the chain stops at the first failing step (a fault, abort, time limit or test
# failure ends the call: nothing more runs on the GPU). Commands are plain shell (env assignments allowed).
# Never copies over pathtracer_gaussiansplatting_amd/libptgs.so: variants are loaded by path
# (GS_LIB=libptgs_<variant>.so, tools/gs_ab_check.py <variant>).
set -uo pipefail
OUT=${1:?out dir}
shift
mkdir -p "$OUT"
sha256sum pathtracer_gaussiansplatting_amd/libptgs*.so > "$OUT/lib_sha256.txt" 2>/dev/null
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for step in "$@"; do
  secs=${step%%|*}
  rest=${step#*|}
  name=${rest%%|*}
  cmd=${rest#*|}
  start=$(date +%s)
  echo "== $name ($secs s): $cmd" | tee -a "$OUT/steps.txt"
  timeout -k 10 "$secs" bash -o pipefail -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "== $name rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a "$OUT/steps.txt"
  tail -n 15 "$OUT/$name.log"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
