#!/usr/bin/env bash
# A/B of fused-attention variants in ONE GPU session: tools/spv_bench.py per library, 3 interleaved rounds.
#   bash tools/spv_ab.sh "base exp_a exp_b"   (base = the default library; others graph-transformer_amd/lib/<name>.so)
set -o pipefail
VARS=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in $VARS; do
    if [ "$v" = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
    U2GNN_HIP_LIB=$L timeout -k 10 120 python tools/spv_bench.py ${SPV_ARGS:-} 2>/dev/null | sed "s/^/$v /" || exit 1
  done
done
