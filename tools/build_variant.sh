#!/usr/bin/env bash
# Build an A/B variant of libu2gnn_hip.so with extra -D flags (kernel experiments):
#   bash tools/build_variant.sh NAME -DFLAG ...   ->  graph-transformer_amd/lib/exp_NAME.so
# then run any tool with U2GNN_HIP_LIB=$PWD/graph-transformer_amd/lib/exp_NAME.so
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/graph-transformer_amd/csrc
B=$(mktemp -d)
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fno-slp-vectorize -I$R/include -I$C -Wall -Wno-unused-function"
pids=()
for f in gemm encoder_ops head_ops window_attn attn_fused small_layer mid_layer; do $H "$@" -c $C/$f.hip -o $B/$f.o & pids+=($!); done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++17 -fPIC -I$R/include -I$C "$@" -c $C/encoder_layer.cpp -o $B/encoder_layer.o
for p in "${pids[@]}"; do wait $p || { echo "build_variant: a compile failed"; rm -rf $B; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/graph-transformer_amd/lib/exp_$NAME.so $B/*.o
rm -rf $B
echo "built exp_$NAME.so"
