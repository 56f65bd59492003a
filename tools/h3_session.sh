#!/usr/bin/env bash
# f16x3 forward policy ("fwdh"): GEMM + native-layer tests, C4 step cost vs fwd6 / bf16x3 (interleaved), 8-seed
# train-mode table, the train-mode parity test.  Usage (via gpurun): bash tools/h3_session.sh TAG
set -o pipefail
TAG=${1:-h3a}
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_gemm_h3_gpu.py tests/test_native_layer_gpu.py -k "h3 or fwdh" \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for p in fwdh fwd6 bf16x3 fwdh fwd6 bf16x3; do
  timeout -k 10 200 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 \
    --neighbors-line 0 --no-roofline --precision $p > gpurun_out/${TAG}_bench_$p.json 2>gpurun_out/${TAG}_bench_$p.err || { tail -20 gpurun_out/${TAG}_bench_$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$p.json'));print('$p', d['ms_per_step'], d['final_loss'])"
done
timeout -k 10 900 python tools/prec_train_probe.py --seeds 987654321,5,11,12,13,14,15,16 --policies ${POLICIES:-fwdh} --fp64 \
  > gpurun_out/${TAG}_prec.jsonl 2> gpurun_out/${TAG}_prec.err || { tail -20 gpurun_out/${TAG}_prec.err; exit 1; }
python - <<PY
import json
for l in open("gpurun_out/${TAG}_prec.jsonl"):
    r = json.loads(l)
    if "policy" in r:
        print(r["seed"], r["policy"], "%.2e" % r["max_err"], r["pass_1e-3"], r.get("relu_flips_vs_oracle32"), r.get("relu_flips_vs_fp64"))
PY
