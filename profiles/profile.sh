#!/bin/bash
# Collect the rocprofv3 evidence for bench.py on a GPU box (run from the repo root via gpurun):
#   pass 1: --kernel-trace --stats                 per-kernel durations (agree with bench.py's HIP events)
#   pass 2: --pmc FETCH_SIZE            (own pass) HBM read side (x2 on gfx950, MI355X_MICROARCH.md §HBM)
#   pass 3: --pmc WRITE_SIZE            (own pass) HBM write side
#   pass 4: --pmc TCC_HIT_sum TCC_MISS_sum         L2 hit rate
#   pass 5: --pmc 8 SQ counters                    VALU issue / lane utilisation, wave wait cycles
# Each pass is its own run (gpurun refuses --pmc with trace domains; counter block limits per pass).
# Outputs under gpurun_out/prof_<tag>/; summarise with profiles/parse_rocprof.py <tag>.
set -euo pipefail
TAG=${1:-r02}
# only the headline legs (C3 path trace, C2 splat): every dispatch of a kernel is the same workload,
# so the per-kernel averages are the per-launch figures bench.py reports
ARGS=${BENCH_ARGS:-"--steps 2 --warmup 1 --headline-only --no-cpu-baseline --no-hybrid --no-gs-1m --no-gs-10m --no-gpu-bvh --no-c1 --no-c5 --no-torus --no-capture"}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
sha256sum pathtracer_gaussiansplatting_amd/libptgs.so > "$OUT/lib_sha256.txt"  # (the profiled library: traffic_latest.json)
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/bench_kt.log" 2>&1
# (counter passes with one frame at a time: under --pmc the front end's stream wait-value packet behind
# the serialised dispatches stalled the frames-in-flight loop (r06); the blend is the same kernel either way)
PARGS="$ARGS --no-splat-overlap"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py $PARGS > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py $PARGS > "$OUT/bench_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d "$OUT/tcc" -o run --output-format csv -- python3 bench.py $PARGS > "$OUT/bench_tcc.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc $SQ -d "$OUT/sq" -o run --output-format csv -- python3 bench.py $PARGS > "$OUT/bench_sq.log" 2>&1
echo "profiles collected in $OUT"
