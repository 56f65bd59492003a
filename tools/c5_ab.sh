# A/B of environment switches on one bench workload (WL = c5 default, c2, c3) in one session:
#   WL=c2 bash tools/c5_ab.sh "BASE VAR=VALUE ..."
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
WL=${WL:-c5}
VARS=${1:-"BASE U2GNN_SPLIT_TARGET=224 U2GNN_SPLIT_TARGET=128 U2GNN_SPLIT_TARGET=896"}
for rep in 1 2; do for v in $VARS; do
E=""; [ "$v" != BASE ] && E=$(echo "$v" | tr ',' ' ')
env $E timeout -k 10 200 python bench.py --workload $WL --steps 30 --warmup 5 --no-roofline --cpu-baseline 0 > gpurun_out/c5ab.json 2>gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5ab.json'));print('$WL $v', d['ms_per_step'], d['value'], d['final_loss'])"
done; done
