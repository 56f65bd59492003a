#!/usr/bin/env bash
# PMC HBM traffic of the current kernels (separate FETCH_SIZE / WRITE_SIZE passes) -> gpurun_out/TAG_pmc_traffic.json
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
bash tools/gpu_pmc.sh "$TAG" || exit 1
F=$(find "$R/gpurun_out/${TAG}_FETCH_SIZE" -name '*.db' | head -1)
W=$(find "$R/gpurun_out/${TAG}_WRITE_SIZE" -name '*.db' | head -1)
python tools/pmc_traffic.py "$F" "$W" gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc_top.txt || exit 1
rm -rf "$R/gpurun_out/${TAG}_FETCH_SIZE" "$R/gpurun_out/${TAG}_WRITE_SIZE"
cat gpurun_out/${TAG}_pmc_top.txt
