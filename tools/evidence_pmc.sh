#!/usr/bin/env bash
# North-star evidence passes (counters only, one rocprofv3 run per pass, no tracing domains besides
# the counters):
#   1. MFMA utilisation of every C4 kernel: SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE (rocprofv3's
#      MfmaUtil = sum(SQ_VALU_MFMA_BUSY_CYCLES) / (GRBM_GUI_ACTIVE per XCD * SIMD_NUM)), node attention
#   2. kernel trace of the neighbour-attention step (where the k+1-slot gather is a real HBM stream)
#   3. FETCH_SIZE / WRITE_SIZE passes of the same neighbour-attention step (gather GB/s)
# Usage (via gpurun): bash tools/evidence_pmc.sh TAG
set -o pipefail
TAG=${1:-ev}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python bench.py --configs 0 --cpu-baseline 0 --no-roofline"
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$R/gpurun_out/${TAG}_MFMA" -o run -- \
    $B --steps 3 --warmup 1 > gpurun_out/${TAG}_MFMA.log 2>&1 || { echo "mfma pass failed"; tail -5 gpurun_out/${TAG}_MFMA.log; exit 1; }
echo "mfma pass done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_nbtrace" -o run -- \
    $B --attention neighbors --steps 4 --warmup 1 > gpurun_out/${TAG}_nbtrace.log 2>&1 || { echo "nb trace failed"; tail -5 gpurun_out/${TAG}_nbtrace.log; exit 1; }
echo "nb trace done"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C -d "$R/gpurun_out/${TAG}_nb_${C}" -o run -- \
      $B --attention neighbors --steps 2 --warmup 1 > gpurun_out/${TAG}_nb_${C}.log 2>&1 || { echo "nb pmc $C failed"; tail -5 gpurun_out/${TAG}_nb_${C}.log; exit 1; }
done
echo "nb pmc done"
M=$(find "$R/gpurun_out/${TAG}_MFMA" -name '*.db' | head -1)
T=$(find "$R/gpurun_out/${TAG}_nbtrace" -name '*.db' | head -1)
F=$(find "$R/gpurun_out/${TAG}_nb_FETCH_SIZE" -name '*.db' | head -1)
W=$(find "$R/gpurun_out/${TAG}_nb_WRITE_SIZE" -name '*.db' | head -1)
python tools/kstats.py "$T" gpurun_out/${TAG}_nb_kstats.txt "$TAG neighbours bench --steps 4 --warmup 1" gpurun_out/${TAG}_nb_ktrace.csv > /dev/null
python tools/pmc_traffic.py "$F" "$W" gpurun_out/${TAG}_nb_pmc_traffic.json > gpurun_out/${TAG}_nb_pmc.log 2>&1 || { tail gpurun_out/${TAG}_nb_pmc.log; exit 1; }
python tools/pmc_mfma.py "$M" gpurun_out/${TAG}_mfma.json > gpurun_out/${TAG}_mfma.txt 2>&1 || { tail gpurun_out/${TAG}_mfma.txt; exit 1; }
cat gpurun_out/${TAG}_mfma.txt
rm -rf "$R/gpurun_out/${TAG}_MFMA" "$R/gpurun_out/${TAG}_nbtrace" "$R/gpurun_out/${TAG}_nb_FETCH_SIZE" "$R/gpurun_out/${TAG}_nb_WRITE_SIZE"
echo "evidence done"
