# x2 GEMM tests (incl. the ping-pong tile codes), then the N^2-product micro-benchmark, then one bench line
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_x2_gpu.py > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -3 gpurun_out/pp_tests.log
XB_CODES=${XB_CODES:-256,130,261,262,263} timeout -k 10 240 python -u tools/x2_bench.py > gpurun_out/pp_bench.log 2>&1 || { cat gpurun_out/pp_bench.log; exit 1; }
cat gpurun_out/pp_bench.log
if [ -n "$PP_BENCH" ]; then timeout -k 10 300 python -u bench.py > gpurun_out/pp_benchline.json 2> gpurun_out/pp_benchline.err || { tail gpurun_out/pp_benchline.err; exit 1; }; cat gpurun_out/pp_benchline.json; fi
