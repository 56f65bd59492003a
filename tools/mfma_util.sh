#!/usr/bin/env bash
# MFMA utilisation of every kernel of the C4 step (one counters-only rocprofv3 pass; tools/pmc_mfma.py).
# Usage (via gpurun): bash tools/mfma_util.sh TAG
set -o pipefail
TAG=${1:-mu}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$R/gpurun_out/${TAG}_MFMA" -o run -- \
    python bench.py --configs 0 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --neighbors-line 0 --no-roofline --steps 3 --warmup 1 > gpurun_out/${TAG}_MFMA.log 2>&1 || { echo "mfma pass failed"; tail -5 gpurun_out/${TAG}_MFMA.log; exit 1; }
M=$(find "$R/gpurun_out/${TAG}_MFMA" -name '*.db' | head -1)
python tools/pmc_mfma.py "$M" gpurun_out/${TAG}_mfma.json > gpurun_out/${TAG}_mfma.txt 2>&1 || { tail gpurun_out/${TAG}_mfma.txt; exit 1; }
cat gpurun_out/${TAG}_mfma.txt
rm -rf "$R/gpurun_out/${TAG}_MFMA"
