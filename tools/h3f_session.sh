#!/usr/bin/env bash
# fwdh with the fused softmax.P.V (f16x3): tests, A/B against the three-pass build (exp_h3unf), the 8-seed
# train-mode table and the train-mode parity test.  Usage (via gpurun): bash tools/h3f_session.sh TAG
set -o pipefail
TAG=${1:-h3f}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_attn_fused_gpu.py tests/test_gemm_h3_gpu.py tests/test_native_layer_gpu.py \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 900 bash tools/ab.sh "base exp_h3unf" > gpurun_out/${TAG}_ab.txt 2>&1 || { tail -20 gpurun_out/${TAG}_ab.txt; exit 1; }
cat gpurun_out/${TAG}_ab.txt
timeout -k 10 200 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 \
  --neighbors-line 0 --no-roofline --precision bf16x3 > gpurun_out/${TAG}_x3.json 2>gpurun_out/${TAG}_x3.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/${TAG}_x3.json'));print('bf16x3', d['ms_per_step'])"
timeout -k 10 900 python tools/prec_train_probe.py --seeds 987654321,5,11,12,13,14,15,16 --policies fwdh --fp64 \
  > gpurun_out/${TAG}_prec.jsonl 2> gpurun_out/${TAG}_prec.err || { tail -20 gpurun_out/${TAG}_prec.err; exit 1; }
python - <<PY
import json
for l in open("gpurun_out/${TAG}_prec.jsonl"):
    r = json.loads(l)
    if "policy" in r and r["policy"] != "oracle_fp32_vs_fp64":
        print(r["seed"], r["policy"], "%.2e" % r["max_err"], r["pass_1e-3"], r.get("relu_flips_vs_oracle32"), r.get("relu_flips_vs_fp64"))
PY
timeout -k 10 600 $T tests/test_train_parity_gpu.py tests/test_unsup_train_parity_gpu.py > gpurun_out/${TAG}_tparity.log 2>&1; tail -3 gpurun_out/${TAG}_tparity.log
