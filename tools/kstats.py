"""Summarise a rocprofv3 kernel trace (rocpd .db -> per-kernel totals).  Usage:
   python tools/kstats.py <run_results.db> [out.txt] [title] [trace_copy.csv]"""
import collections
import csv
import os
import subprocess
import sys
import tempfile

db = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else None
title = sys.argv[3] if len(sys.argv) > 3 else ""
tmp = tempfile.mkdtemp()
subprocess.run(["rocpd2csv", "-i", db, "-d", tmp], check=True, capture_output=True)
rows = list(csv.DictReader(open(os.path.join(tmp, "out_kernel_trace.csv"))))
if len(sys.argv) > 4:   # keep the raw trace (timeline analysis: tools/timeline.py)
    import shutil
    shutil.copy(os.path.join(tmp, "out_kernel_trace.csv"), sys.argv[4])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
lines = [title, "share   total_ms  calls   avg_us  kernel"]
for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1]):
    lines.append(f"{t / tot * 100:5.1f}% {t / 1e3:9.2f} {c:6d} {t / c:8.1f}  {n[:160]}")
lines.append(f"total_kernel_ms {tot / 1e3:.2f}")
txt = "\n".join(lines) + "\n"
if out:
    open(out, "w").write(txt)
print(txt)
