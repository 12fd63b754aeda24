# r03: f2 Gram staging rewrite -- f2 tests, masked ASIS bench + kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_masked.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_f2_tests.log 2>&1 || { tail -30 gpurun_out/r03_f2_tests.log; exit 1; }
tail -1 gpurun_out/r03_f2_tests.log
rm -rf gpurun_out/r03_f2_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_f2_prof -o run --output-format csv -- python3 bench.py --workload masked_asis --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_f2_prof.log 2>&1 || { tail -20 gpurun_out/r03_f2_prof.log; exit 1; }
grep -v "^\[" gpurun_out/r03_f2_prof.log | tail -1 | cut -c1-200
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_f2_prof -name run_kernel_stats.csv | head -1)")" > gpurun_out/r03_f2_kstats.txt; grep -E "f2_|synth_blocks|sht_" gpurun_out/r03_f2_kstats.txt
