"""Per-stream idle gaps of a rocprofv3 kernel trace (the CSV tools/kstats.py keeps) over the last N
steps (Adam kernels mark step ends): the busiest stream's gaps > 3 us, grouped by the kernel pair
around them.  Usage: python tools/stream_gaps.py trace.csv [steps]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
key = next(k for k in ("Stream_Id", "Queue_Id", "Stream_ID") if k in rows[0])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key], r["Kernel_Name"]) for r in rows)
ends = [e for s, e, q, n in ev if "adam" in n]
t0, t1 = ends[-steps - 1], ends[-1]
win = [(s, e, q, n) for s, e, q, n in ev if s >= t0 and e <= t1]
busy = collections.Counter()
for s, e, q, n in win:
    busy[q] += e - s
main = busy.most_common(1)[0][0]
m = [(s, e, n) for s, e, q, n in win if q == main]


def short(n):
    return re.sub(r"\(anonymous namespace\)::", "", n)[:60]


gaps = collections.defaultdict(lambda: [0, 0.0])
for (s0, e0, n0), (s1, e1, n1) in zip(m, m[1:]):
    g = (s1 - e0) / 1e3
    if g > 3:
        k = (short(n0), short(n1))
        gaps[k][0] += 1
        gaps[k][1] += g
print(f"step {(t1 - t0) / 1e6 / steps:.3f} ms; stream {main} busy {busy[main] / 1e6 / steps:.3f} ms/step; "
      f"its gaps > 3 us: {sum(v[1] for v in gaps.values()) / steps:.1f} us/step")
for k, v in sorted(gaps.items(), key=lambda x: -x[1][1])[:10]:
    print(f"{v[1] / steps:7.1f} us/step {v[0] / steps:4.1f}x  {k[0]} -> {k[1]}")
