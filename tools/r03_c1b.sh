set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_c1b_tests.log 2>&1 || { tail -30 gpurun_out/r03_c1b_tests.log; exit 1; }
tail -1 gpurun_out/r03_c1b_tests.log
timeout -k 10 300 python -u tools/step_ab.py centered 512 256 1 200 GS_CENTERED_FUSED=1 GS_CENTERED_NONE=1 > gpurun_out/r03_c1b_ab.log 2>&1 || { tail -20 gpurun_out/r03_c1b_ab.log; exit 1; }
cat gpurun_out/r03_c1b_ab.log
