#!/usr/bin/env bash
# Kernel trace of the C4 bench under an environment switch (e.g. U2GNN_OVERLAP=0), for main-stream gap
# analysis with tools/stream_gaps.py.  Usage (via gpurun): bash tools/gap_prof.sh TAG [VAR=VALUE ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
env "$@" GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/${TAG}_p" -o run -- python bench.py --configs 0 --steps 10 --warmup 3 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_p.log 2>&1 || { tail -5 gpurun_out/${TAG}_p.log; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_p" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/stream_gaps.py gpurun_out/${TAG}_ktrace.csv 5
rm -rf "$R/gpurun_out/${TAG}_p"
