#!/usr/bin/env bash
# SQ counters for the GEMM micro-benchmark, one rocprofv3 --pmc pass per counter (counters only, no
# tracing domains).  Usage: GB_ONLY="QK^T,dV" bash tools/gemm_pmc.sh TAG [prec]
set -o pipefail
TAG=${1:-gpmc}
PREC=${2:-bf16x3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp GB_REPS=${GB_REPS:-5}
for C in SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS \
         SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM \
         SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_SALU TA_BUSY_avr; do
  timeout -k 10 120 rocprofv3 --pmc $C -d "$R/gpurun_out/${TAG}/${C}" -o run -- python tools/gemm_bench.py $PREC \
      > gpurun_out/${TAG}_${C}.log 2>&1 || { echo "pmc $C failed"; tail -3 gpurun_out/${TAG}_${C}.log; }
done
echo pmc done
