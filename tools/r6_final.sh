#!/usr/bin/env bash
# Round-6 final measurement of the current build, in the order the bench line's lookups need them: GPU tests; the
# C4 kernel trace (the line's rocprof fields); the PMC FETCH_SIZE / WRITE_SIZE passes (its traffic fields); the
# C5 / C2 / C3 kernel traces (their lines' largest kernels) -- each summary copied into profiles/r06 on the box
# first, where bench.py finds it by this build's source id -- then the bench line with the CPU baseline, and
# smoke().  Every GPU step under its own time limit; the first failure ends the script.
# Usage (via gpurun): bash tools/r6_final.sh TAG
set -o pipefail
TAG=${1:-r6f}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out profiles/r06; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> gpurun_out/${TAG}_tests.log; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit 1
PCMD="python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --configs 0"
GPU_MAX_HW_QUEUES=8 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof" -o run -- $PCMD > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/${TAG}_prof.log; exit 1; }
DB=$(find "$R/gpurun_out/${TAG}_prof" -name '*.db' | head -1)
python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG $PCMD (rocprofv3 --kernel-trace --stats)" gpurun_out/${TAG}_ktrace.csv > /dev/null || exit 1
python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt || exit 1
rm -rf "$R/gpurun_out/${TAG}_prof"
echo "c4 trace done"
bash tools/gpu_pmc.sh $TAG || exit 1
F=$(find "$R/gpurun_out/${TAG}_FETCH_SIZE" -name '*.db' | head -1)
W=$(find "$R/gpurun_out/${TAG}_WRITE_SIZE" -name '*.db' | head -1)
python tools/pmc_traffic.py "$F" "$W" gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc.log 2>&1 || { tail gpurun_out/${TAG}_pmc.log; exit 1; }
rm -rf "$R/gpurun_out/${TAG}_FETCH_SIZE" "$R/gpurun_out/${TAG}_WRITE_SIZE"
echo "pmc done"
for WL in c5 c2 c3; do
  bash tools/wl_trace.sh ${TAG}_$WL $WL > gpurun_out/${TAG}_${WL}_trace.log 2>&1 || { tail -5 gpurun_out/${TAG}_${WL}_trace.log; exit 1; }
done
echo "workload traces done"
cp gpurun_out/${TAG}_kstats.json gpurun_out/${TAG}_pmc_traffic.json gpurun_out/${TAG}_c5_kstats.json \
   gpurun_out/${TAG}_c2_kstats.json gpurun_out/${TAG}_c3_kstats.json profiles/r06/ || exit 1
timeout -k 10 900 python bench.py --steps 30 --warmup 5 --cpu-baseline 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
echo "bench done"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
