mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_x2_gpu.py > gpurun_out/x2_tests.log 2>&1; rc=$?
tail -25 gpurun_out/x2_tests.log
if [ $rc -eq 0 ]; then timeout -k 10 200 python -u tools/x2_bench.py > gpurun_out/x2_bench.log 2>&1; echo bench rc=$?; cat gpurun_out/x2_bench.log; fi
