#!/usr/bin/env bash
# A/B kernel variants in ONE GPU session (box-to-box clock differences are ~5-7 %):
#   bash tools/ab.sh "base exp_oldloop exp_nosb" [GB_ONLY shapes]
# WL=c2 (or c5 / c3): the bench line of that workload instead of C4
# PROBE=1: the C4 line with the bench's live dS probe on (as in BENCH) and its average launch time printed
# base = the default library; others = graph-transformer_amd/lib/<name>.so.  Each variant runs
# the GEMM micro-benchmark (optional shapes) and bench.py twice, interleaved.
set -o pipefail
VARS=$1
ONLY=${2:-}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in $VARS; do
    if [ "$v" = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
    if [ -n "$ONLY" ] && [ $rep = 1 ]; then
      U2GNN_HIP_LIB=$L GB_ONLY="$ONLY" timeout -k 10 200 python tools/gemm_bench.py bf16x3 2>/dev/null | sed "s/^/$v /" || exit 1
    fi
    if [ -n "${WL:-}" ]; then
      U2GNN_HIP_LIB=$L timeout -k 10 200 python bench.py --workload $WL --steps 30 --warmup 5 --cpu-baseline 0 --neighbors-line 0 > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
    else
    NR=--no-roofline; [ -n "${PROBE:-}" ] && NR=""
    U2GNN_HIP_LIB=$L timeout -k 10 200 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --neighbors-line 0 $NR > gpurun_out/ab_$v.json 2>gpurun_out/ab_$v.err || exit 1
    fi
    python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));r=d.get('roofline') or {};print('$v', 'step_ms', d['ms_per_step'], d['final_loss'], 'probe_us', r.get('avg_launch_us'))"
  done
done
