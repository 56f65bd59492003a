#!/usr/bin/env bash
# Quick GPU iteration: gpu tests -> C4 bench (no CPU baseline) -> C5 bench [-> C5 kernel trace if PROF5=1].
# Usage (via gpurun): bash tools/gpu_quick.sh TAG
set -o pipefail
TAG=${1:-q}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${NOTESTS:-0}" != "1" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/${TAG}_c4.json 2> gpurun_out/${TAG}_c4.err || { tail -20 gpurun_out/${TAG}_c4.err; exit 1; }
cat gpurun_out/${TAG}_c4.json
timeout -k 10 300 python bench.py --workload c5 --steps 30 --warmup 5 > gpurun_out/${TAG}_c5.json 2> gpurun_out/${TAG}_c5.err || { tail -20 gpurun_out/${TAG}_c5.err; exit 1; }
cat gpurun_out/${TAG}_c5.json
if [ "${PROF5:-0}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_p5" -o run -- python bench.py --workload c5 --steps 10 --warmup 2 --no-roofline > gpurun_out/${TAG}_p5.log 2>&1 || exit 1
DB=$(find "$R/gpurun_out/${TAG}_p5" -name '*.db' | head -1)
[ -n "$DB" ] && python tools/kstats.py "$DB" gpurun_out/${TAG}_c5_kstats.txt "$TAG bench.py --workload c5 --steps 10 --warmup 2" gpurun_out/${TAG}_c5_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_c5_ktrace.csv 5 > gpurun_out/${TAG}_c5_timeline.txt
rm -rf "$R/gpurun_out/${TAG}_p5"
fi
