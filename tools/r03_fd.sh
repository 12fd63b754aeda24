# r03: statistics finish + C_l draw in one launch (k_finish_draw) -- targeted tests, full suite, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread -k "centered" > gpurun_out/r03_fd_t0.log 2>&1 || { grep -n "PASSED\|FAILED" gpurun_out/r03_fd_t0.log | tail -3; tail -15 gpurun_out/r03_fd_t0.log; exit 1; }
tail -1 gpurun_out/r03_fd_t0.log
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_fd_tests.log 2>&1 || { grep -n "PASSED\|FAILED" gpurun_out/r03_fd_tests.log | tail -3; tail -15 gpurun_out/r03_fd_tests.log; exit 1; }
tail -1 gpurun_out/r03_fd_tests.log
GS_AB_NOSTORE=1 timeout -k 10 300 python3 -u tools/step_ab.py centered 512 256 1 500 GS_CLS_PRE=0 GS_FINISH_DRAW_OFF=1 GS_CLS_PRE=1 > gpurun_out/r03_fd_ab.log 2>&1 || { tail -20 gpurun_out/r03_fd_ab.log; exit 1; }
cat gpurun_out/r03_fd_ab.log
