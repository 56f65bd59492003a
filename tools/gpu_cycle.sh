#!/usr/bin/env bash
# One GPU iteration: gpu tests -> bench (with CPU baseline unless NOCPU=1) -> rocprofv3 kernel trace of
# the SAME bench command (its dS average must agree with the bench line's live roofline timing).
# GPU_MAX_HW_QUEUES=8 is set in front of rocprofv3 itself: u2gnn_hip.ensure_hw_queues sets it at import,
# which is too late under rocprofv3 (its preloaded library initialises HIP before the program runs).
# Usage (via gpurun): bash tools/gpu_cycle.sh TAG
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${NOTESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit 1
fi
CPU=1; [ "${NOCPU:-0}" = "1" ] && CPU=0
CMD="python bench.py --steps 30 --warmup 5 --cpu-baseline $CPU"
timeout -k 10 600 $CMD > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
# the profiled run: the same timed region, without the CPU baseline and the extra lines after it (fp32, on-the-fly
# pipeline), so the trace holds the timed steps' launches (and their averages match the bench line's probe)
PCMD="python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --configs 0"
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- $PCMD > gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
[ -n "$DB" ] && python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG $PCMD (rocprofv3 --kernel-trace --stats)" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
find "$R/gpurun_out/${TAG}_prof" -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
rm -rf "$R/gpurun_out/${TAG}_prof"
