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
    # beside the text: per-kernel and per-(kernel, grid) averages tagged with the native build id, which bench.py
    # cites (rocprof_stats) when the build matches -- the grid split separates launches of one kernel at
    # different sizes (the gather of a batch's slot-0 rows vs the bench's all-slot gather roofline)
    import json
    import re
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd"))
    from u2gnn_hip._lib import source_build_id

    def short(n):
        n = re.sub(r"^void ", "", n)
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        return n.split("(")[0] if "<" not in n else n[:n.index(">") + 1]
    grid = collections.defaultdict(lambda: [0, 0.0])
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g = grid[(short(r["Kernel_Name"]), int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0))]
        g[0] += 1
        g[1] += d
    js = {"title": title, "build_id": source_build_id(), "total_kernel_ms": tot / 1e3,
          "kernels": {short(n): {"calls": c, "avg_us": t / c, "total_ms": t / 1e3} for n, (c, t) in agg.items()},
          "by_grid": [{"kernel": k, "grid": gx, "calls": c, "avg_us": t / c} for (k, gx), (c, t) in
                      sorted(grid.items(), key=lambda kv: -kv[1][1])[:80]]}
    json.dump(js, open(os.path.splitext(out)[0] + ".json", "w"), indent=1)
print(txt)
