#!/usr/bin/env bash
# A/B library variants on one workload in ONE GPU session, REPS interleaved rounds:
#   bash tools/ab_wl.sh "base exp_r4" c4 [REPS]
# base = the default library; others = graph-transformer_amd/lib/<name>.so.
set -o pipefail
VARS=$1; WL=${2:-c4}; REPS=${3:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in $(seq $REPS); do
  for v in $VARS; do
    if [ "$v" = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
    U2GNN_HIP_LIB=$L timeout -k 10 200 python bench.py --workload $WL --steps 30 --warmup 5 --cpu-baseline 0 --no-roofline > gpurun_out/ab_${WL}_$v.json 2>gpurun_out/ab_${WL}_$v.err || { tail -3 gpurun_out/ab_${WL}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab_${WL}_$v.json'));print('$WL', '$v', 'step_ms', d['ms_per_step'], d['final_loss'])"
  done
done
