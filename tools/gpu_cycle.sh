#!/usr/bin/env bash
# One GPU iteration: gpu tests -> bench (with CPU baseline unless NOCPU=1) -> rocprofv3 kernel trace.
# Usage (via gpurun): bash tools/gpu_cycle.sh TAG
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ "${NOTESTS:-0}" != "1" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/${TAG}_tests.log 2>&1
echo "tests rc=$?" >> gpurun_out/${TAG}_tests.log
tail -3 gpurun_out/${TAG}_tests.log
fi
CPU=1; [ "${NOCPU:-0}" = "1" ] && CPU=0
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --cpu-baseline $CPU > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
[ -n "$DB" ] && python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG bench.py --steps 10 --warmup 2" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
find "$R/gpurun_out/${TAG}_prof" -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
rm -rf "$R/gpurun_out/${TAG}_prof"
