#!/usr/bin/env bash
# SQ / TCC counters of the whole small-width layer (tools/small_layer_bench.py, C5 shape), one rocprofv3 --pmc pass per
# counter (counters only, no tracing domains), then the per-kernel table.  Usage: bash tools/sl_pmc.sh TAG
set -o pipefail
TAG=${1:-slpmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp SLB_SHAPES=1
timeout -k 10 120 python tools/small_layer_bench.py > gpurun_out/$TAG/bench.txt 2>&1 || { echo "bench failed"; cat gpurun_out/$TAG/bench.txt; exit 1; }
cat gpurun_out/$TAG/bench.txt
for C in GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM \
         SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU \
         SQ_ACTIVE_INST_LDS SQ_INSTS_SALU FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$R/gpurun_out/$TAG/$C" -o run -- python tools/small_layer_bench.py 3 \
      > gpurun_out/$TAG/$C.log 2>&1 || { echo "pmc $C failed"; tail -3 gpurun_out/$TAG/$C.log; exit 1; }
done
python tools/pmc_table.py gpurun_out/$TAG > gpurun_out/$TAG/table.txt 2>&1
cat gpurun_out/$TAG/table.txt
find gpurun_out/$TAG -name '*.db' -delete
