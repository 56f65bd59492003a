#!/usr/bin/env bash
# HBM traffic per kernel: two separate rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE cannot share a
# pass on gfx950's TCC slots), no tracing domains besides the counters.  Usage: bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  GPU_MAX_HW_QUEUES=8 timeout -s KILL 300 rocprofv3 --pmc $C -d "$R/gpurun_out/${TAG}_${C}" -o run -- python bench.py --configs 0 --steps 3 --warmup 1 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_${C}.log 2>&1 || { echo "pmc $C failed"; tail -5 gpurun_out/${TAG}_${C}.log; exit 1; }
done
echo pmc done
