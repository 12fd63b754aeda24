# r03: MH timeline + default bench line after the MH rewrite
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
GIBBS_HIP_LIB=gibbssampler_amd/libgibbs_hip_timeline.so timeout -k 10 200 python -u tools/mh_timeline.py > gpurun_out/r03_tl.log 2>&1 || { tail -20 gpurun_out/r03_tl.log; exit 1; }
cat gpurun_out/r03_tl.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_mh2_tests.log 2>&1 || { tail -30 gpurun_out/r03_mh2_tests.log; exit 1; }
tail -1 gpurun_out/r03_mh2_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_mh2_bench.json 2> gpurun_out/r03_mh2_bench.err || { tail -20 gpurun_out/r03_mh2_bench.err; exit 1; }
cat gpurun_out/r03_mh2_bench.json
