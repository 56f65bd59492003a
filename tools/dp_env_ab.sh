#!/usr/bin/env bash
# Same-session A/B of torch ProcessGroupNCCL watchdog settings on the one-rank data-parallel overhead (C4). Usage (via gpurun): bash tools/dp_env_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
OUT=gpurun_out/dpenv.txt; : > $OUT
E0=""
E1="TORCH_NCCL_ENABLE_MONITORING=0 TORCH_NCCL_ASYNC_ERROR_HANDLING=0 TORCH_NCCL_DUMP_ON_TIMEOUT=0"
for rep in 1 2; do
  for m in nodist none none_env overlap overlap_env; do
    case $m in nodist) A=""; E="$E0";; none) A="--force-dist --allreduce none"; E="$E0";; none_env) A="--force-dist --allreduce none"; E="$E1";;
      overlap) A="--force-dist --allreduce overlap"; E="$E0";; overlap_env) A="--force-dist --allreduce overlap"; E="$E1";; esac
    env $E timeout -k 10 200 python bench.py --configs 0 --neighbors-line 0 $A --steps 40 --warmup 5 --cpu-baseline 0 --no-roofline --fp32-steps 0 --pipeline-steps 0 > gpurun_out/dpe_$m.json 2> gpurun_out/dpe_$m.err || { tail -5 gpurun_out/dpe_$m.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/dpe_$m.json'));print('rep $rep', '$m', d['ms_per_step'], d['host_issue_ms_per_step'])" | tee -a $OUT
  done
done
