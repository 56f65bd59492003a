#!/usr/bin/env bash
# Round-6 session A: affected GPU tests, bf16x6 GEMM timings, fwd6 kernel trace, precision variants (8 seeds)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k signed_ds tests/test_train_parity_gpu.py tests/test_unsup_train_parity_gpu.py \
  tests/test_graph_replay_gpu.py tests/test_attn_small_gpu.py tests/test_small_layer_gpu.py tests/test_dp_gloo_gpu.py \
  > gpurun_out/r6a_tests.log 2>&1 || { tail -40 gpurun_out/r6a_tests.log; exit 1; }
tail -2 gpurun_out/r6a_tests.log
bash tools/x6_gemm.sh || exit 1
bash tools/prof_prec.sh x6a fwd6 || exit 1
timeout -k 10 900 python tools/prec_train_probe.py --seeds 987654321,5,11,12,13,14,15,16 --policies x6_nopv,x6_noqk --fp64 \
  > gpurun_out/x6_prec2.jsonl 2> gpurun_out/x6_prec2.err || { tail -20 gpurun_out/x6_prec2.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/x6_prec2.jsonl"):
    r = json.loads(l)
    if "policy" in r:
        print(r["seed"], r["policy"], "%.2e" % r["max_err"], r["pass_1e-3"], r.get("relu_flips_vs_oracle32"), r.get("relu_flips_vs_fp64"))
PY
