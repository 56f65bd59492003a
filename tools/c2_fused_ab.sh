#!/usr/bin/env bash
# C2 (IMDBBINARY, Np = 128) with the three-pass attention forward (base: fused only from Np >= 1024) against the
# fused form at every row count (exp_fusedall), both policies, one session.  Usage (via gpurun): bash tools/c2_fused_ab.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_native_layer_gpu.py \
  > gpurun_out/c2ab_tests.log 2>&1 || { tail -30 gpurun_out/c2ab_tests.log; exit 1; }
tail -1 gpurun_out/c2ab_tests.log
for rep in 1 2; do
  for v in base exp_fusedall; do
    if [ "$v" = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
    for p in fwdh bf16x3; do
      U2GNN_HIP_LIB=$L timeout -k 10 200 python bench.py --workload c2 --steps 30 --warmup 5 --cpu-baseline 0 \
        --precision $p > gpurun_out/c2ab_${v}_$p.json 2>gpurun_out/c2ab_${v}_$p.err || { tail -5 gpurun_out/c2ab_${v}_$p.err; exit 1; }
      python -c "import json;d=json.load(open('gpurun_out/c2ab_${v}_$p.json'));print('$v', '$p', d['ms_per_step'])"
    done
  done
done
