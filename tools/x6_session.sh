#!/usr/bin/env bash
# Round-6 session: the bf16x6 ("fwd6") forward policy -- kernel tests, the 8-seed train-mode precision table, and the
# C4 step cost against bf16x3 / fwd32 in one session.  Output under gpurun_out/x6_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gemm_x6_gpu.py > gpurun_out/x6_tests.log 2>&1 || { tail -30 gpurun_out/x6_tests.log; exit 1; }
tail -2 gpurun_out/x6_tests.log
timeout -k 10 400 $T tests/test_native_layer_gpu.py -k "fwd6 or fwd32" > gpurun_out/x6_native.log 2>&1 || { tail -30 gpurun_out/x6_native.log; exit 1; }
tail -2 gpurun_out/x6_native.log
for p in ${PRECS:-bf16x3 fwd6 bf16x3 fwd6}; do
  timeout -k 10 200 python bench.py --configs 0 --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 \
    --no-roofline --precision $p > gpurun_out/x6_bench_$p.json 2>gpurun_out/x6_bench_$p.err || { tail -20 gpurun_out/x6_bench_$p.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/x6_bench_$p.json'));print('$p', d['ms_per_step'], d['final_loss'])"
done
if [ -n "${PROBE_SEEDS:-}" ]; then
  timeout -k 10 900 python tools/prec_train_probe.py --seeds "$PROBE_SEEDS" --policies "${POLICIES:-x6_proj,x6_all}" --fp64 \
    > gpurun_out/x6_prec.jsonl 2> gpurun_out/x6_prec.err || { tail -20 gpurun_out/x6_prec.err; exit 1; }
  python - <<'EOF'
import json
for l in open("gpurun_out/x6_prec.jsonl"):
    r = json.loads(l)
    if "policy" in r:
        print(r["seed"], r["policy"], "%.2e" % r["max_err"], r["pass_1e-3"], r.get("relu_flips_vs_oracle32"), r.get("relu_flips_vs_fp64"))
EOF
fi
