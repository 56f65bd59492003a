# neighbour-mode A/B of environment switches (one session): bash tools/nb_ab.sh "BASE VAR=VAL ..."
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
for rep in 1 2; do for v in $1; do
E=""; [ "$v" != BASE ] && E=$(echo "$v" | tr ',' ' ')
env $E timeout -k 10 300 python bench.py --attention neighbors --steps 10 --warmup 2 --cpu-baseline 0 --no-roofline > gpurun_out/nbab.json 2>gpurun_out/nbab.err || { tail -5 gpurun_out/nbab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/nbab.json'));print('$v', d['ms_per_step'], d['value'], d['final_loss'])"
done; done
