#!/usr/bin/env bash
# Round-end measurement: final_cycle (GPU tests, C4 bench + CPU baseline, rocprof summary, PMC traffic),
# the C5 / C2 / C3 bench lines and smoke().  Usage (via gpurun): bash tools/round_final.sh TAG
set -o pipefail
TAG=${1:-final}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/final_cycle.sh $TAG || exit 1
for W in c5 c2 c3; do
  timeout -k 10 300 python bench.py --workload $W --steps 30 --warmup 5 > gpurun_out/${TAG}_$W.json 2> gpurun_out/${TAG}_$W.err || { tail -5 gpurun_out/${TAG}_$W.err; exit 1; }
  cut -c1-200 gpurun_out/${TAG}_$W.json
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
