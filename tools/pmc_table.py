"""Per-kernel average of every counter collected by tools/gemm_pmc.sh.
Usage: python tools/pmc_table.py gpurun_out/TAG"""
import collections
import csv
import glob
import os
import subprocess
import sys
import tempfile


def main(root):
    rows = collections.defaultdict(dict)
    for db in sorted(glob.glob(os.path.join(root, "*", "**", "*.db"), recursive=True)):
        tmp = tempfile.mkdtemp()
        subprocess.run(["rocpd2csv", "-i", db, "-d", tmp], check=True, capture_output=True)
        for path in glob.glob(os.path.join(tmp, "*counter_collection*.csv")):
            acc = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(path)):
                k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("((")[0]
                acc[(k, r["Counter_Name"])][r.get("Dispatch_Id") or r.get("Correlation_Id")] += float(r["Counter_Value"])
            for (k, c), d in acc.items():
                rows[k][c] = sum(d.values()) / len(d)
    cols = sorted({c for v in rows.values() for c in v})
    for k, v in rows.items():
        print(k)
        for c in cols:
            if c in v:
                print(f"    {c:28s} {v[c]:16.4g}")


if __name__ == "__main__":
    main(sys.argv[1])
