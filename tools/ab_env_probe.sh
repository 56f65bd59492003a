#!/usr/bin/env bash
# tools/ab_env.sh with the bench's live dominant-kernel probe on: per variant the step time and the dS
# (or --probe) launch time inside the timed region.  Usage: bash tools/ab_env_probe.sh "BASE U2GNN_X=1" [args]
set -o pipefail
VARS=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-3}); do
  for v in $VARS; do
    E=""; [ "$v" != BASE ] && E=$(echo "$v" | tr ',' ' ')
    env $E timeout -k 10 200 python bench.py --steps 40 --warmup 5 --cpu-baseline 0 "$@" > gpurun_out/abprobe.json 2>gpurun_out/abprobe.err || { tail -5 gpurun_out/abprobe.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abprobe.json'));r=d['roofline'];print('$v', 'step_ms', d['ms_per_step'], d['value'], 'probe_us', r.get('avg_launch_us'), 'frac', r.get('frac'))"
  done
done
