set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload c5 --steps 30 --warmup 5 > gpurun_out/c5a_bench.json 2> gpurun_out/c5a_bench.err || { tail -20 gpurun_out/c5a_bench.err; exit 1; }
cat gpurun_out/c5a_bench.json
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/c5a_prof" -o run -- python bench.py --workload c5 --steps 10 --warmup 2 --no-roofline > gpurun_out/c5a_prof.log 2>&1
echo "prof rc=$?"
DB=$(find "$R/gpurun_out/c5a_prof" -name '*.db' | head -1)
[ -n "$DB" ] && python tools/kstats.py "$DB" gpurun_out/c5a_kstats.txt "c5a bench.py --workload c5 --steps 10 --warmup 2" gpurun_out/c5a_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/c5a_ktrace.csv 5 > gpurun_out/c5a_timeline.txt
rm -rf "$R/gpurun_out/c5a_prof"
