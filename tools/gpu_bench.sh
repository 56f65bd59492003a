set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err || exit 1
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof1 -o run -- python bench.py --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/prof1.log 2>&1
echo done
