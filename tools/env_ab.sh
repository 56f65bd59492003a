#!/usr/bin/env bash
# A/B of a runtime environment setting, one session, interleaved: bench lines of the given workloads
# with and without it.  Usage (via gpurun): bash tools/env_ab.sh "VAR=value" "c5 c2 c3 c4"
set -o pipefail
SETTING=$1; WLS=${2:-"c5 c2 c3 c4"}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
for rep in 1 2; do
  for w in $WLS; do
    for mode in off on; do
      if [ $w = c4 ]; then A="--configs 0 --fp32-steps 0 --pipeline-steps 0 --no-roofline"; else A="--workload $w"; fi
      if [ $mode = on ]; then E="env $SETTING"; else E=""; fi
      timeout -k 10 200 $E python bench.py $A --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/envab.json 2>/dev/null || exit 1
      python -c "import json;d=json.load(open('gpurun_out/envab.json'));print('$w', '$mode', d['ms_per_step'], d.get('final_loss'))"
    done
  done
done
