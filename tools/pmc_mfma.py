"""MFMA utilisation per kernel from one rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE pass
(tools/evidence_pmc.sh).

rocprofv3's derived MfmaUtil (counter_defs.yaml) = sum(SQ_VALU_MFMA_BUSY_CYCLES) /
(GRBM_GUI_ACTIVE per XCD * SIMD_NUM).  rocprofv3 reports GRBM_GUI_ACTIVE summed over the 8 XCDs
(MI355X_MICROARCH.md, DVFS note), so the kernel's cycles are GRBM_GUI_ACTIVE / 8; SIMD_NUM = 256 CUs
x 4 SIMDs = 1024.  SQ_VALU_MFMA_BUSY_CYCLES counts 32 cycles per v_mfma_f32_32x32x16_bf16, so 100 %
means every SIMD's matrix pipe busy on every cycle of the kernel.  For the bf16x3 GEMMs three MFMAs
carry one algorithmic product, so algorithmic throughput = util * 2.5 PF * (clock / 2.4 GHz) / 3.
Usage: python tools/pmc_mfma.py <run_results.db> <out.json>
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

XCDS, SIMDS = 8, 1024


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    return name.split("(")[0] if "<" not in name else name[:name.index(">") + 1]


def main():
    tmp = tempfile.mkdtemp()
    subprocess.run(["rocpd2csv", "-i", sys.argv[1], "-d", tmp], check=True, capture_output=True)
    path = glob.glob(os.path.join(tmp, "*counter_collection*.csv"))[0]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(path)):
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        names[key] = short(r["Kernel_Name"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for key, c in per.items():
        a = agg[names[key]]
        a[0] += 1
        a[1] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[2] += c.get("GRBM_GUI_ACTIVE", 0.0)
    out = {"method": "util = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (GRBM_GUI_ACTIVE/8 * 1024); one --pmc pass over "
                     "bench.py --steps 3 --warmup 1 (C4, bf16x3)", "kernels": {}}
    tot_busy = tot_cyc = 0.0
    for k, (n, busy, gui) in agg.items():
        cyc = gui / XCDS
        tot_busy += busy
        tot_cyc += cyc
        out["kernels"][k] = {"launches": n, "mfma_busy_cycles_per_launch": busy / n,
                             "kernel_cycles_per_launch": cyc / n,
                             "mfma_util": busy / (cyc * SIMDS) if cyc > 0 else 0.0}
    out["all_kernels_mfma_util"] = tot_busy / (tot_cyc * SIMDS) if tot_cyc > 0 else 0.0
    json.dump(out, open(sys.argv[2], "w"), indent=1)
    print("mfma_util  cycles/launch  launches  kernel")
    for k, v in sorted(out["kernels"].items(), key=lambda kv: -kv[1]["kernel_cycles_per_launch"] * kv[1]["launches"])[:24]:
        print(f"{v['mfma_util'] * 100:8.1f}%  {v['kernel_cycles_per_launch']:12.0f}  {v['launches']:8d}  {k}")
    print(f"all kernels (cycle-weighted): {out['all_kernels_mfma_util'] * 100:.1f}%")


if __name__ == "__main__":
    main()
