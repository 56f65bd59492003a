# gather variant A/B (tools/gather_ab.py) + the gather tests, on the GPU box
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gather" > gpurun_out/ga_test.log 2>&1
for m in ${GA_MODES:-0 2}; do U2GNN_GATHER_MODE=$m GA_CEIL=${GA_CEIL:-} timeout -k 10 120 python -u tools/gather_ab.py >> gpurun_out/ga.log 2>&1; GA_CEIL=; done
grep -v amdgpu.ids gpurun_out/ga.log; tail -1 gpurun_out/ga_test.log
