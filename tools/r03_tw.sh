# r03: sweep shape A/B (4 tiles x 1 chunk vs 2 tiles x 2 chunks with LDS pair sums) at configs[2]
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_tw_tests.log 2>&1 || { tail -30 gpurun_out/r03_tw_tests.log; exit 1; }
tail -1 gpurun_out/r03_tw_tests.log
GS_SWEEP_TW=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_tw2_tests.log 2>&1 || { tail -30 gpurun_out/r03_tw2_tests.log; exit 1; }
tail -1 gpurun_out/r03_tw2_tests.log
timeout -k 10 300 python -u tools/step_ab.py noncentered 1024 512 32 50 GS_SWEEP_TW=4 GS_SWEEP_TW=2 > gpurun_out/r03_tw_ab.log 2>&1 || { tail -20 gpurun_out/r03_tw_ab.log; exit 1; }
cat gpurun_out/r03_tw_ab.log
timeout -k 10 300 python -u tools/step_ab.py noncentered 1024 512 32 50 GS_SWEEP_TW=2 GS_SWEEP_TW=4 > gpurun_out/r03_tw_ab2.log 2>&1 || { tail -20 gpurun_out/r03_tw_ab2.log; exit 1; }
cat gpurun_out/r03_tw_ab2.log
