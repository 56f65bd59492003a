#!/usr/bin/env bash
# Kernel summary + timeline of one bench workload (c2 / c3 / c5) under rocprofv3.
# Usage (via gpurun): bash tools/wl_prof.sh TAG WORKLOAD
set -o pipefail
TAG=$1; WL=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_p" -o run -- python bench.py --workload $WL --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_p.log 2>&1 || { tail -5 gpurun_out/${TAG}_p.log; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_p" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG bench.py --workload $WL --steps 10 --warmup 2" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
rm -rf "$R/gpurun_out/${TAG}_p"
head -25 gpurun_out/${TAG}_kstats.txt | cut -c1-150; head -4 gpurun_out/${TAG}_timeline.txt
