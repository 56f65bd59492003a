#!/usr/bin/env bash
# Round-6 session B: the fused bf16x6 attention forward -- tests, C4 step cost vs bf16x3, kernel trace, 8-seed table
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_attn_fused_gpu.py tests/test_gemm_x6_gpu.py "tests/test_native_layer_gpu.py" -k "bf16x6 or x6 or fwd6" \
  > gpurun_out/r6b_tests.log 2>&1 || { tail -40 gpurun_out/r6b_tests.log; exit 1; }
tail -2 gpurun_out/r6b_tests.log
timeout -k 10 600 $T tests/test_train_parity_gpu.py -k "fwd6 or bf16x3" > gpurun_out/r6b_tparity.log 2>&1 || tail -3 gpurun_out/r6b_tparity.log
tail -2 gpurun_out/r6b_tparity.log
for p in bf16x3 fwd6 bf16x3 fwd6; do
  timeout -k 10 200 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 \
    --no-roofline --precision $p > gpurun_out/r6b_bench_$p.json 2>gpurun_out/r6b_bench_$p.err || { tail -20 gpurun_out/r6b_bench_$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/r6b_bench_$p.json'));print('$p', d['ms_per_step'], d['final_loss'])"
done
bash tools/prof_prec.sh x6b fwd6 || exit 1
timeout -k 10 900 python tools/prec_train_probe.py --seeds 987654321,5,11,12,13,14,15,16 --policies fwd6 --fp64 \
  > gpurun_out/x6_prec3.jsonl 2> gpurun_out/x6_prec3.err || { tail -20 gpurun_out/x6_prec3.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/x6_prec3.jsonl"):
    r = json.loads(l)
    if "policy" in r:
        print(r["seed"], r["policy"], "%.2e" % r["max_err"], r["pass_1e-3"], r.get("relu_flips_vs_oracle32"), r.get("relu_flips_vs_fp64"))
PY
