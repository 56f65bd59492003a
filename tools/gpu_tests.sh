#!/usr/bin/env bash
# Targeted GPU check: the given test files (all failures listed), then one short C4 bench line.
# Stops at a crash / timeout.  Usage (via gpurun): bash tools/gpu_tests.sh TAG tests/a.py tests/b.py ...
set -o pipefail
TAG=${1:-quick}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest "$@" -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc" >> $O/tests.log
grep -E "FAILED|ERROR|passed|failed" $O/tests.log | tail -25
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 ${C4ARGS:-} > $O/c4.json 2> $O/c4.err \
  || { echo "c4 failed rc=$?"; tail -8 $O/c4.err; exit 1; }
cat $O/c4.json
exit $rc
