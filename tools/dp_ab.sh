#!/usr/bin/env bash
# Same-session A/B of the data-parallel overhead at one rank (C4): no process group / 1-rank RCCL group with no
# all-reduce / the overlapped all-reduce (native RCCL, round 6) / the same through c10d / bucketed after the
# backward, interleaved, REPS reps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/${TAG:-dpab}.txt; : > $OUT
for rep in $(seq 1 ${REPS:-2}); do
  for m in nodist none overlap overlap_c10d after; do
    E=""
    case $m in nodist) A="";; overlap_c10d) A="--force-dist --allreduce overlap"; E="U2GNN_NATIVE_RCCL=0";; *) A="--force-dist --allreduce $m";; esac
    env $E timeout -k 10 200 python bench.py --configs 0 $A --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline --fp32-steps 0 --pipeline-steps 0 > gpurun_out/dpab_$m.json 2> gpurun_out/dpab_$m.err || { tail -20 gpurun_out/dpab_$m.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/dpab_$m.json'));print('rep $rep', '$m', d['ms_per_step'], d['final_loss'], d['host_issue_ms_per_step'], d['config']['parallelism'])" | tee -a $OUT
  done
done
