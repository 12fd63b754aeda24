# r03: small-map SHT changes -- SHT + masked tests, masked ASIS and PCG kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py tests/test_gpu_tt.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_sht_tests.log 2>&1 || { tail -30 gpurun_out/r03_sht_tests.log; exit 1; }
tail -1 gpurun_out/r03_sht_tests.log
rm -rf gpurun_out/r03_sht_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_sht_prof -o run --output-format csv -- python3 bench.py --workload masked_asis --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_sht_prof.log 2>&1 || { tail -20 gpurun_out/r03_sht_prof.log; exit 1; }
grep -h '"metric"' gpurun_out/r03_sht_prof.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('masked_asis', d['value'], d['ms_per_step'])"
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_sht_prof -name run_kernel_stats.csv | head -1)")" > gpurun_out/r03_sht_kstats.txt; grep -E "sht_|f2_" gpurun_out/r03_sht_kstats.txt
