set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
PCMD="python bench.py --steps 30 --warmup 5 --cpu-baseline 0 --fp32-steps 0 --pipeline-steps 0 --configs 0"
for v in ${VARS:-base exp_probenf}; do
  if [ $v = base ]; then L=""; else L="$R/graph-transformer_amd/lib/$v.so"; fi
  U2GNN_HIP_LIB=$L GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pp_$v" -o run -- $PCMD > gpurun_out/pp_$v.json 2> gpurun_out/pp_$v.err || exit 1
  DB=$(find "$R/gpurun_out/pp_$v" -name '*.db' | head -1)
  python tools/kstats.py "$DB" gpurun_out/pp_${v}_kstats.txt "$v $PCMD" gpurun_out/pp_${v}_ktrace.csv > /dev/null && python tools/timeline.py gpurun_out/pp_${v}_ktrace.csv 5 > gpurun_out/pp_${v}_timeline.txt
  rm -rf "$R/gpurun_out/pp_$v" gpurun_out/pp_${v}_ktrace.csv
  python -c "import json;d=json.load(open('gpurun_out/pp_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], 'probe_us', r['avg_launch_us'])"
  grep -m1 "2, 2, 32, false, true, 7" gpurun_out/pp_${v}_kstats.txt
done
