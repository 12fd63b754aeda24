# r03: full GPU suite + default bench + kernel stats of the default bench + rows A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_full_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_full_tests.log; exit 1; }
tail -1 gpurun_out/r03_full_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_full_bench.json 2> gpurun_out/r03_full_bench.err || { tail -20 gpurun_out/r03_full_bench.err; exit 1; }
cat gpurun_out/r03_full_bench.json
rm -rf gpurun_out/r03_full_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_full_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-every 20 > gpurun_out/r03_full_prof.log 2>&1 || { tail -20 gpurun_out/r03_full_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_full_prof -name run_kernel_stats.csv | head -1)")"
timeout -k 10 300 python -u tools/step_ab.py noncentered 1024 512 32 50 GS_SWEEP_ROWS=16 GS_SWEEP_ROWS=12 GS_SWEEP_ROWS=20 > gpurun_out/r03_rows_ab.log 2>&1 || { tail -20 gpurun_out/r03_rows_ab.log; exit 1; }
cat gpurun_out/r03_rows_ab.log
