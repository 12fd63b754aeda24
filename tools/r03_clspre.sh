# r03: C_l variates drawn by extra workgroups of the latency-form sweep -- tests + A/B + configs[1] bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u -m pytest tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_clspre_tests0.log 2>&1 || { tail -30 gpurun_out/r03_clspre_tests0.log; exit 1; }
tail -1 gpurun_out/r03_clspre_tests0.log
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_clspre_tests.log 2>&1 || { tail -30 gpurun_out/r03_clspre_tests.log; exit 1; }
tail -1 gpurun_out/r03_clspre_tests.log
GS_AB_NOSTORE=1 timeout -k 10 300 python3 -u tools/step_ab.py centered 512 256 1 500 GS_CLS_PRE=0 GS_CLS_PRE=1 > gpurun_out/r03_clspre_ab.log 2>&1 || { tail -20 gpurun_out/r03_clspre_ab.log; exit 1; }
cat gpurun_out/r03_clspre_ab.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --time-every 100 > gpurun_out/r03_clspre_c2.json 2> gpurun_out/r03_clspre_c2.err || { tail -20 gpurun_out/r03_clspre_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_clspre_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
