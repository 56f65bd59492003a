#!/usr/bin/env bash
# Kernel summaries of the C4 bench under rocprofv3 for several environment variants (one GPU session).
# Usage (via gpurun): bash tools/ab_prof.sh TAG "BASE U2GNN_X=0 ..."
set -o pipefail
TAG=$1; VARS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for v in $VARS; do
  E=""; [ "$v" != BASE ] && E=$(echo "$v" | tr ',' ' ')
  env $E GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_${i}_p" -o run -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/${TAG}_${i}.log 2>&1 || { tail -5 gpurun_out/${TAG}_${i}.log; exit 1; }
  DB=$(find "$R/gpurun_out/${TAG}_${i}_p" -name '*.db' | head -1)
  python tools/kstats.py "$DB" gpurun_out/${TAG}_${i}_kstats.txt "$TAG [$v] bench.py --steps 10 --warmup 2" > /dev/null || exit 1
  rm -rf "$R/gpurun_out/${TAG}_${i}_p"
  echo "== $v"; head -30 gpurun_out/${TAG}_${i}_kstats.txt | cut -c1-140
  i=$((i+1))
done
