#!/usr/bin/env bash
# Cheaper staging splits (fp16: two mixed-precision fmas per element; bf16: packed residual subtraction), same bits:
# kernel tests, C4 A/B against the previous build (exp_oldsplit), and the policies' losses of one bench run.
# Usage (via gpurun): bash tools/split_session.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gemm_h3_gpu.py tests/test_gemm_x6_gpu.py tests/test_kernels_gpu.py tests/test_attn_fused_gpu.py \
  tests/test_native_layer_gpu.py > gpurun_out/split_tests.log 2>&1 || { tail -40 gpurun_out/split_tests.log; exit 1; }
tail -1 gpurun_out/split_tests.log
timeout -k 10 900 bash tools/ab.sh "base exp_oldsplit" > gpurun_out/split_ab.txt 2>&1 || { tail -20 gpurun_out/split_ab.txt; exit 1; }
cat gpurun_out/split_ab.txt
timeout -k 10 400 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --pipeline-steps 0 --neighbors-line 0 \
  --no-roofline > gpurun_out/split_bench.json 2> gpurun_out/split_bench.err || { tail -20 gpurun_out/split_bench.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/split_bench.json'));print('fwdh', d['ms_per_step'], d['final_loss'], {k:(d[k]['ms_per_step'], d[k]['final_loss']) for k in ('bf16x3','fwd6','fwd32','fp32')})"
