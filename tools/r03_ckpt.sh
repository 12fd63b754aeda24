# r03: checkpoint / resume tests + graph suite
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_graph.py tests/test_gpu_surface.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_ckpt_tests.log 2>&1 || { tail -30 gpurun_out/r03_ckpt_tests.log; exit 1; }
tail -1 gpurun_out/r03_ckpt_tests.log
