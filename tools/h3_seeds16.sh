#!/usr/bin/env bash
# 16-seed train-mode table of the fp32-class forward policies (fwdh fused / three-pass, fwd6, fwd32) on the C4 batch.
# Usage (via gpurun): bash tools/h3_seeds16.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
S=987654321,5,11,12,13,14,15,16,17,18,19,20,21,22,23,24
timeout -k 10 1000 python -u tools/prec_train_probe.py --seeds $S --policies fwdh,fwdh_3pass,fwd6,fwd32 --fp64 \
  > gpurun_out/seeds16.jsonl 2> gpurun_out/seeds16.err || { tail -20 gpurun_out/seeds16.err; exit 1; }
python - <<'PY'
import json, collections
agg = collections.defaultdict(lambda: [0, 0, 0, []])
for l in open("gpurun_out/seeds16.jsonl"):
    r = json.loads(l)
    if "policy" not in r:
        continue
    a = agg[r["policy"]]
    a[0] += 1
    a[1] += int(r["pass_1e-3"])
    f = r.get("relu_flips_vs_oracle32") or r.get("relu_flips_vs_fp64") or [0]
    a[3].append(f[0])
for k, (n, ok, _, fl) in agg.items():
    print(f"{k:22s} seeds {n:2d} within 1e-3: {ok:2d}  flips/step {min(fl)}-{max(fl)} total {sum(fl)}")
PY
