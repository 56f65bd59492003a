"""Per-stream, per-kernel us/step of two kernel traces side by side (tools/kstats.py CSV copies), over
each trace's final N optimizer steps.  Usage: python tools/trace_cmp.py a.csv b.csv [steps]"""
import collections
import csv
import re
import sys


def load(path, steps):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows)
    ends = [e for s, e, q, n in ev if "adam_kernel" in n]
    t0, t1 = ends[-steps - 1], ends[-1]
    agg = collections.defaultdict(float)
    for s, e, q, n in ev:
        if s >= t0 and e <= t1:
            nm = re.sub(r"\(anonymous namespace\)::|void ", "", n).split("(")[0][:70]
            agg[(q, nm)] += (e - s) / 1e3 / steps
    return agg, (t1 - t0) / 1e3 / steps


steps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
a, ta = load(sys.argv[1], steps)
b, tb = load(sys.argv[2], steps)
print(f"step us: {ta:9.1f} {tb:9.1f}")
for k in sorted(set(a) | set(b), key=lambda k: (k[0], -max(a.get(k, 0), b.get(k, 0)))):
    x, y = a.get(k, 0.0), b.get(k, 0.0)
    if max(x, y) >= 5:
        print(f"{k[0]:>3} {x:9.1f} {y:9.1f} {y - x:+8.1f}  {k[1]}")
