#!/usr/bin/env bash
# rocprofv3 kernel trace + per-kernel summary of one C5 (or C2 / C3) bench run.  Usage (via gpurun):
#   bash tools/c5_prof.sh TAG [c5|c2|c3]
set -o pipefail
TAG=${1:-c5}
W=${2:-c5}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- \
  python bench.py --workload $W --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG bench.py --workload $W --steps 10 --warmup 2" > /dev/null
rm -rf "$R/gpurun_out/${TAG}_prof"
