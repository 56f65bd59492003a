#!/usr/bin/env bash
# C4 step: eager vs HIP-graph replay, kernel trace of each (per-kernel durations + idle gaps).
# Usage (via gpurun): bash tools/graph_ab.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-gab}; shift
R=${GRAPH_AB_ROOT:-${GRAFT_REPO_ROOT:-$(pwd)}}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for g in 0 1; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_g$g" -o run -- python bench.py --configs ${CFG:-0} --graph $g --steps 10 --warmup 3 --cpu-baseline 0 --no-roofline "$@" > gpurun_out/${TAG}_g$g.json 2> gpurun_out/${TAG}_g$g.err || { tail -20 gpurun_out/${TAG}_g$g.err; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_g$g" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_g${g}_kstats.txt "$TAG graph=$g" gpurun_out/${TAG}_g${g}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_g${g}_ktrace.csv 5 > gpurun_out/${TAG}_g${g}_timeline.txt || exit 1
rm -rf "$R/gpurun_out/${TAG}_g$g"
done
