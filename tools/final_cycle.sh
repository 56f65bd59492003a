#!/usr/bin/env bash
# Full measurement of the current build: gpu tests -> bench (CPU baseline) -> rocprof kernel trace
# -> PMC HBM traffic table (separate FETCH_SIZE / WRITE_SIZE passes).  Usage: bash tools/final_cycle.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_cycle.sh $TAG || exit 1
bash tools/gpu_pmc.sh $TAG || exit 1
F=$(find "$R/gpurun_out/${TAG}_FETCH_SIZE" -name '*.db' | head -1)
W=$(find "$R/gpurun_out/${TAG}_WRITE_SIZE" -name '*.db' | head -1)
python tools/pmc_traffic.py "$F" "$W" gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc.log 2>&1 || { tail gpurun_out/${TAG}_pmc.log; exit 1; }
rm -rf "$R/gpurun_out/${TAG}_FETCH_SIZE" "$R/gpurun_out/${TAG}_WRITE_SIZE"
echo "pmc table written"
