"""HBM traffic per GEMM kernel instance from two rocprofv3 --pmc passes (tools/gpu_pmc.sh).

hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024, averaged over the kernel's launches:
FETCH_SIZE / WRITE_SIZE are in KB; on gfx950 FETCH_SIZE counts exactly half of the bytes of a wide
(16 B/lane) coalesced read (MI355X_MICROARCH.md, HBM section) — the GEMM operand loads are
16 B/lane float4 loads, hence x2; WRITE_SIZE is exact for streaming stores.  Infinity-Cache hits
are counted as fetches.  Usage:
    python tools/pmc_traffic.py <FETCH run_results.db> <WRITE run_results.db> <out.json>
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys
import tempfile


def per_kernel(db, counter):
    tmp = tempfile.mkdtemp()
    subprocess.run(["rocpd2csv", "-i", db, "-d", tmp], check=True, capture_output=True)
    path = glob.glob(os.path.join(tmp, "*counter_collection*.csv"))[0]
    agg = collections.defaultdict(lambda: [0, 0.0])
    seen = set()
    grids = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
        name = re.sub(r"^void ", "", r["Kernel_Name"])
        name = re.sub(r"\(anonymous namespace\)::", "", name)
        name = name.split("((")[0].split("(")[0] if "<" not in name else name[:name.index(">") + 1]
        g = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
        for nm in (name, f"{name}@grid={g}"):   # per kernel, and per kernel and launch size
            a = agg[nm]
            if (key, nm) not in seen:
                a[0] += 1
                seen.add((key, nm))
            a[1] += float(r["Counter_Value"])
        grids[name].add(g)
    # the largest launch size of each kernel under a fixed name (bench.py: the gather roofline's launches)
    for name, gs in grids.items():
        if len(gs) > 1:
            agg[f"{name}@maxgrid"] = agg[f"{name}@grid={max(gs)}"]
    return agg


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd"))
    from u2gnn_hip._lib import source_build_id
    out = {"method": "(2*FETCH_SIZE + WRITE_SIZE) KB * 1024 per launch; separate --pmc passes; "
                     "bench.py --steps 3 --warmup 1 (C4 COLLAB-like, bf16x3)",
           "build_id": source_build_id(), "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        nf, f = fetch.get(k, [0, 0.0])
        nw, w = write.get(k, [0, 0.0])
        if nf == 0 or nw == 0:
            continue
        out["kernels"][k] = {"launches": nf, "fetch_kb_per_launch": f / nf, "write_kb_per_launch": w / nw,
                             "hbm_bytes_per_launch": round((2 * f / nf + w / nw) * 1024)}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:12]:
        print(f"{v['hbm_bytes_per_launch'] / 1e6:10.2f} MB/launch  n={v['launches']:4d}  {k}")


if __name__ == "__main__":
    main()
