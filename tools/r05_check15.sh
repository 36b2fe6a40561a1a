#!/bin/bash
# round-5 GPU step: fused front end with 128 / 64 Gaussians per workgroup (shorter per-workgroup chain);
# bit-exactness, static + moving A/B, then the splat tests against the 128 library (copied over
# libptgs.so in this box's scratch copy)
set -uo pipefail
O=gpurun_out/r05v; mkdir -p $O
timeout -k 10 120 python3 tools/gs_ab_check.py f128 > $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py f128 >> $O/check.log 2>&1 || exit 1
GS_SORTED=2 timeout -k 10 120 python3 tools/gs_ab_check.py f64 >> $O/check.log 2>&1 || exit 1
GS_AB_ROUNDS=3 timeout -k 10 300 bash tools/gs_ab.sh "" "GS_LIB=libptgs_f128.so" "GS_LIB=libptgs_f64.so" > $O/ab.log 2>&1 || exit 1
AB_ROUNDS=3 timeout -k 10 300 python3 tools/gs_orbit_ab.py base f128 f64 > $O/orbit_ab.log 2>&1 || exit 1
cp pathtracer_gaussiansplatting_amd/libptgs_f128.so pathtracer_gaussiansplatting_amd/libptgs.so || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider -k "gaussian or splat or tight or raster or hybrid or c4 or c5 or dist" > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/pytest.log
exit 0
