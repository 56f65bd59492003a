#!/usr/bin/env bash
# x2 GEMM ablations in one GPU session: bash tools/x2_ab.sh "base exp_x2NOLOAD ..." [codes]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for v in $1; do
  if [ "$v" = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
  echo "== $v"
  U2GNN_HIP_LIB=$L XB_CODES=${2:-256,130} timeout -k 10 200 python tools/x2_bench.py 2>/dev/null | grep -v "^softmax\|^total" || exit 1
done
