#!/usr/bin/env bash
# Kernel trace + summary of the C4 bench line at one precision policy: bash tools/prof_prec.sh TAG PREC
set -o pipefail
TAG=$1; PREC=${2:-bf16x3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
PCMD="python bench.py --steps 20 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --configs 0 --no-roofline --precision $PREC"
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- $PCMD > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG $PCMD (rocprofv3 --kernel-trace --stats)" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
rm -rf "$R/gpurun_out/${TAG}_prof"
head -30 gpurun_out/${TAG}_kstats.txt
