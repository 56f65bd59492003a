#!/usr/bin/env bash
# bf16x6 vs bf16x3 device time of the forward products at the C4 shapes (tools/gemm_bench.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for p in bf16x3 bf16x6; do
  GB_ONLY="QK^T,P.V   ,QKVb,FFN1d,outpr,FFN2r" timeout -k 10 200 python tools/gemm_bench.py $p > gpurun_out/x6_gemm_$p.txt 2>&1 || { tail -5 gpurun_out/x6_gemm_$p.txt; exit 1; }
  cat gpurun_out/x6_gemm_$p.txt
done
