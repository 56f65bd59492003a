#!/usr/bin/env bash
# Interleaved A/B of bench.py argument sets / environments in ONE GPU session, REPS rounds (default 3):
#   bash tools/ab_args.sh "BASE|--no-roofline|ENV:U2GNN_OVERLAP=0"
# Each variant is "|"-separated: BASE = defaults, ENV:K=V[,K=V] = environment, anything else = bench args.
set -o pipefail
IFS='|' read -ra VARS <<< "$1"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for v in "${VARS[@]}"; do
    E=""; A=""
    if [ "$v" != BASE ]; then
      if [[ "$v" == ENV:* ]]; then E=$(echo "${v#ENV:}" | tr ',' ' '); else A="$v"; fi
    fi
    env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-baseline 0 $A > gpurun_out/abargs.json 2>gpurun_out/abargs.err || { tail -5 gpurun_out/abargs.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abargs.json'));r=d.get('roofline') or {};print('$v'.ljust(32), 'step_ms', d['ms_per_step'], d['value'], 'dS_us', r.get('avg_launch_us'))"
  done
done
