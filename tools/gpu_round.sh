#!/bin/bash
# One gpurun call that gathers a round's evidence in order, stopping at the first failure:
#   1. tools/gpu_check.sh <tag>        GPU tests, smoke, bench (the driver's round-end tiers)
#   2. tools/gs_bands.sh               tile-row band kernel traces (C2, 10M at 4K)       [GS_BANDS_RUN=1]
#   3. profiles/profile.sh <tag>       kernel trace + separate PMC passes of the bench   [PROFILE_RUN=1]
# Logs under gpurun_out/ (check_<tag>/, gsb_*/, prof_<tag>/).
set -uo pipefail
TAG=${1:-r04}
bash tools/gpu_check.sh "$TAG" || exit $?
if [ "${GS_BANDS_RUN:-1}" = "1" ]; then
  bash tools/gs_bands.sh > gpurun_out/gs_bands_${TAG}.log 2>&1 || exit $?
fi
if [ "${PROFILE_RUN:-1}" = "1" ]; then
  bash profiles/profile.sh "$TAG" || exit $?
fi
echo "gpu_round $TAG done"
