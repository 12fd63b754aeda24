# r03: SHT prefetch default -- SHT + masked GPU tests, masked C5 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_pfv_tests.log 2>&1 || { tail -20 gpurun_out/r03_pfv_tests.log; exit 1; }
tail -1 gpurun_out/r03_pfv_tests.log
timeout -k 10 400 python3 -u bench.py --workload masked > gpurun_out/r03_pfv_c5.json 2> gpurun_out/r03_pfv_c5.err || { tail -20 gpurun_out/r03_pfv_c5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_pfv_c5.json')); print(d['value'], d['ms_per_step'], d['roofline'])"
