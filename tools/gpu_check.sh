#!/bin/bash
# The driver's round-end GPU tiers, rehearsed on one gpurun box (run from the repo root):
#   1. pytest -m gpu (durations)   2. __graft_entry__.smoke()   3. bench.py --gpus 1 --steps 20 --warmup 5
# Each step has its own time limit and the chain stops at the first failure. Logs under
# gpurun_out/check_<tag>/; tools/gpu_check_summary.py turns them into profiles/<tag>_gputest.txt and
# profiles/<tag>_bench.json.
set -uo pipefail
TAG=${1:-r03}
OUT=gpurun_out/check_${TAG}
mkdir -p "$OUT"
sha256sum pathtracer_gaussiansplatting_amd/libptgs.so > "$OUT/lib_sha256.txt"
start=$(date +%s)
timeout -k 10 840 python -u -m pytest tests -m gpu -q --durations=40 --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?
echo "pytest rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a "$OUT/pytest.log"
[ $rc -eq 0 ] || exit $rc
start=$(date +%s)
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?
echo "smoke rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a "$OUT/smoke.log"
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = "1" ] && exit 0
start=$(date +%s)
timeout -k 10 590 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.log" 2> "$OUT/bench.err"
rc=$?
echo "bench rc=$rc wall=$(( $(date +%s) - start ))s" | tee -a "$OUT/bench.err"
exit $rc
