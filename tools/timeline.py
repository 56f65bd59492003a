"""Timeline view of a rocprofv3 kernel trace (the CSV tools/kstats.py keeps): GPU busy time (union of
kernel intervals), per-stream busy time, time with both streams busy, and the idle gaps, over the
window from the first to the last kernel of the trace's final N steps (adam_kernel marks a step end),
optionally ending SKIP steps before the trace's last one (bench.py's pipeline_rate steps follow the timed
region: --pipeline-steps 20 plus 2 warmup steps = skip 22).
Usage: python tools/timeline.py trace.csv [steps] [skip]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
key = next(k for k in ("Stream_Id", "Queue_Id", "Stream_ID") if k in rows[0])
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r[key], r["Kernel_Name"]) for r in rows)
ends = [e for s, e, q, n in ev if "adam_kernel" in n or "adam_dev_kernel" in n]
if len(ends) < steps + skip + 1:
    sys.exit(f"only {len(ends)} optimizer steps in the trace")
t0, t1 = ends[len(ends) - skip - steps - 1], ends[len(ends) - skip - 1]
win = [(max(s, t0), min(e, t1), q, n) for s, e, q, n in ev if e > t0 and s < t1]


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    return tot + ((cur_e - cur_s) if cur_e is not None else 0)


span = t1 - t0
busy = union([(s, e) for s, e, q, n in win])
print(f"window {steps} steps: {span / 1e6 / steps:.3f} ms/step; GPU busy {busy / 1e6 / steps:.3f} ms/step "
      f"({busy / span * 100:.1f}%), idle {(span - busy) / 1e6 / steps:.3f} ms/step")
qs = sorted({q for s, e, q, n in win})
per = {q: union([(s, e) for s, e, qq, n in win if qq == q]) for q in qs}
for q in qs:
    cnt = sum(1 for w in win if w[2] == q)
    print(f"  stream {q}: busy {per[q] / 1e6 / steps:.3f} ms/step, {cnt / steps:.0f} kernels/step")
if len(qs) > 1:
    both = sum(per.values()) - busy
    print(f"  overlap (>=2 streams busy): {both / 1e6 / steps:.3f} ms/step")
gaps = []
last = None
for s, e, q, n in sorted(win):
    if last is not None and s > last[0]:
        gaps.append((s - last[0], last[1], n))
    if last is None or e > last[0]:
        last = (e, n)
gaps.sort(reverse=True)
print(f"idle gaps: {len(gaps) / steps:.0f}/step, total {sum(g[0] for g in gaps) / 1e6 / steps:.3f} ms/step; largest:")
for g, a, b in gaps[:8]:
    print(f"  {g / 1e3:7.1f} us  after {a[:70]}  before {b[:70]}")
