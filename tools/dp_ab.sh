#!/usr/bin/env bash
# Same-session A/B of the data-parallel overhead at one rank (C4): no process group / 1-rank RCCL group with no
# all-reduce / the overlapped all-reduce / bucketed after the backward, interleaved, REPS reps; QUEUES="8 16":
# each with that many HIP hardware queues (GPU_MAX_HW_QUEUES).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-dpab}.txt; : > $OUT
for rep in $(seq 1 ${REPS:-2}); do
 for q in ${QUEUES:-8}; do
  for m in ${MODES:-nodist none overlap after}; do
    case $m in nodist) A="";; *) A="--force-dist --allreduce $m";; esac
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --configs 0 $A --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline --fp32-steps 0 --pipeline-steps 0 > gpurun_out/dpab_$m.json 2> gpurun_out/dpab_$m.err || { tail -20 gpurun_out/dpab_$m.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/dpab_$m.json'));print('rep $rep', 'queues $q', '$m', d['ms_per_step'], d['final_loss'], d['host_issue_ms_per_step'], d['config']['parallelism'])" | tee -a $OUT
  done
 done
done
