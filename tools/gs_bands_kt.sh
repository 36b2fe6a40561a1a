set -euo pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for b in 0 3 7; do
  GS_CFG=10m GS_BAND=balanced:$b timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r06o/b$b -o run --output-format csv -- python3 tools/gs_bands.py > gpurun_out/r06o/b$b.log 2>&1
  grep "ms/frame" gpurun_out/r06o/b$b.log
done
