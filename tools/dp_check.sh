#!/usr/bin/env bash
# DP path on one GPU: bench.py with a 1-rank RCCL group (--force-dist), all-reduce modes A/B,
# plus a kernel trace of the overlapped mode.  Usage (via gpurun): bash tools/dp_check.sh TAG
set -o pipefail
TAG=${1:-dp}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
for m in ${MODES:-none after overlap}; do
timeout -k 10 200 python bench.py --configs 0 --force-dist --allreduce $m --graph ${GRAPH:--1} --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_$m.json 2> gpurun_out/${TAG}_$m.err || { tail -20 gpurun_out/${TAG}_$m.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_$m.json'));print('$m', d['ms_per_step'], d['value'], d['final_loss'], d['config']['parallelism'])"
done
timeout -k 10 200 python bench.py --configs 0 --graph ${GRAPH:--1} --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_nodist.json 2>/dev/null && python -c "import json;d=json.load(open('gpurun_out/${TAG}_nodist.json'));print('nodist', d['ms_per_step'], d['value'])"
[ "${NOPROF:-0}" = "1" ] && exit 0
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_p" -o run -- python bench.py --configs 0 --force-dist --allreduce overlap --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_p.log 2>&1 || exit 1
DB=$(find "$R/gpurun_out/${TAG}_p" -name '*.db' | head -1)
[ -n "$DB" ] && python tools/kstats.py "$DB" gpurun_out/${TAG}_kstats.txt "$TAG force-dist overlap" gpurun_out/${TAG}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/${TAG}_ktrace.csv 5 > gpurun_out/${TAG}_timeline.txt
rm -rf "$R/gpurun_out/${TAG}_p"
