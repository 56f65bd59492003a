set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for rep in 1 2; do for v in BASE U2GNN_SPLIT_TARGET=224 U2GNN_SPLIT_TARGET=128 U2GNN_SPLIT_TARGET=896; do
E=""; [ "$v" != BASE ] && E=$v
env $E timeout -k 10 200 python bench.py --workload c5 --steps 30 --warmup 5 --no-roofline > gpurun_out/c5ab.json 2>gpurun_out/c5ab.err || { tail -5 gpurun_out/c5ab.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/c5ab.json'));print('C5 $v', d['ms_per_step'], d['value'], d['final_loss'])"
done; done
