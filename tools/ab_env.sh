#!/usr/bin/env bash
# A/B environment switches in ONE GPU session, interleaved, REPS rounds (default 3):
#   bash tools/ab_env.sh "BASE U2GNN_DV_SIDE=1 U2GNN_MAIN_PRIO=1,U2GNN_DV_SIDE=1" [extra bench args]
set -o pipefail
VARS=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    E=""; [ "$v" != BASE ] && E=$(echo "$v" | tr ',' ' ')
    env $E timeout -k 10 200 python bench.py --configs 0 --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline "$@" > gpurun_out/abenv.json 2>gpurun_out/abenv.err || { tail -5 gpurun_out/abenv.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abenv.json'));print('$v', 'step_ms', d['ms_per_step'], d['value'], d['final_loss'], 'host', d.get('host_issue_ms_per_step'))"
  done
done
