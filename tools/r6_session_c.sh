#!/usr/bin/env bash
# Round-6 session C: fwd6 (unfused x6 attention) parity tests, then the full default bench line (fwd6) beside bf16x3
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $T tests/test_train_parity_gpu.py tests/test_native_layer_gpu.py -k "fwd6" > gpurun_out/r6c_tests.log 2>&1 || { tail -30 gpurun_out/r6c_tests.log; exit 1; }
tail -2 gpurun_out/r6c_tests.log
timeout -k 10 500 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --pipeline-steps 0 > gpurun_out/r6c_bench.json 2> gpurun_out/r6c_bench.err || { tail -20 gpurun_out/r6c_bench.err; exit 1; }
timeout -k 10 500 python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --pipeline-steps 0 --fp32-steps 0 --precision bf16x3 > gpurun_out/r6c_bench_x3.json 2> gpurun_out/r6c_bench_x3.err || { tail -20 gpurun_out/r6c_bench_x3.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r6c_bench.json", "gpurun_out/r6c_bench_x3.json"):
    d = json.load(open(f))
    print(f, d["dtype"], d["ms_per_step"], d["value"])
    r = d.get("roofline") or {}
    print("  ds", r.get("avg_launch_us"), r.get("frac"), "step_frac", r.get("step_frac"))
    for k, v in (r.get("other_kernels") or {}).items():
        print("  ", k, v["kernel"][:60], v["avg_launch_us"], v["frac"])
    for k in ("fp32", "fwd32", "bf16x3", "fwd6"):
        if k in d: print("  ", k, d[k]["ms_per_step"])
    for k in ("c5", "c2", "c3"):
        if k in d: print("  ", k, d[k]["ms_per_step"], (d[k].get("roofline") or {}).get("frac"))
    g = d.get("gather") or {}
    print("  gather", g.get("frac"), g.get("avg_launch_us"), g.get("traffic"))
PY
