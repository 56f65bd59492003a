#!/usr/bin/env bash
# Affected GPU tests, then the full GPU suite, then the latency-bound bench lines (C5, C2, C3) and C4.
# Usage (via gpurun): bash tools/gpu_quick_c5.sh TAG
set -o pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "reduce_batch or gemm_group" -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_new_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_new_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
for W in c5 c2 c3 c4; do
  timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/${TAG}_$W.json 2> gpurun_out/${TAG}_$W.err || { tail -5 gpurun_out/${TAG}_$W.err; exit 1; }
  cut -c1-260 gpurun_out/${TAG}_$W.json
done
