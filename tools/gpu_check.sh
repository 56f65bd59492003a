#!/usr/bin/env bash
# GPU check of a build: the -m gpu suite (all failures listed, not -x), then short C4 / C5 bench lines
# and the 1-rank RCCL path of the C5 data-parallel step (--force-dist).  Stops at a crash / timeout.
# Usage (via gpurun): bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-chk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python -u bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "$n failed rc=$?"; tail -8 $O/$n.err; exit 1; }
  echo "== $n"; cat $O/$n.json
}
run c4 300 --steps 30 --warmup 5 --cpu-baseline 0 ${C4ARGS:-}
run c5 300 --workload c5 --steps 30 --warmup 5 --cpu-baseline 0
run c5dist 300 --workload c5 --force-dist --steps 20 --warmup 3 --cpu-baseline 0 --no-roofline
exit $rc
