#!/usr/bin/env bash
# Kernel trace of one bench workload (c5 / c2 / c3): rocprof summary + per-step timeline.
# Usage (via gpurun): bash tools/wl_trace.sh TAG WORKLOAD [extra bench args]
set -o pipefail
TAG=${1:-wl}; W=${2:-c2}; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_p" -o run -- python bench.py --workload $W --steps 20 --warmup 3 --cpu-baseline 0 "$@" > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || { tail -20 gpurun_out/${TAG}.err; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_p" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG $W" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
rm -rf "$R/gpurun_out/${TAG}_p"
