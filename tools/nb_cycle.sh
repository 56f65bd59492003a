#!/usr/bin/env bash
# Neighbour-attention iteration: window/gather kernel tests -> neighbours bench -> kernel trace.
# Usage (via gpurun): bash tools/nb_cycle.sh TAG
set -o pipefail
TAG=${1:-nb}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_neighbors_gpu.py \
    tests/test_kernels_gpu.py -k "window or neighbors or gather" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --attention neighbors --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline \
    > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -5 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- \
    python bench.py --attention neighbors --steps 4 --warmup 1 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG neighbours bench --steps 4 --warmup 1" gpurun_out/${TAG}_ktrace.csv > /dev/null
python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 3 > gpurun_out/${TAG}_timeline.txt
head -8 gpurun_out/${TAG}_kstats.txt
rm -rf "$R/gpurun_out/${TAG}_prof"
