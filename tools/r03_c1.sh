# r03: configs[1] (centered TEB, N_side 256, L 512, 1 chain): tests, A/B of sweep shapes, bench, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_c1_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_c1_tests.log; exit 1; }
tail -1 gpurun_out/r03_c1_tests.log
timeout -k 10 300 python -u tools/step_ab.py centered 512 256 1 200 GS_CENTERED_UNFUSED=1 GS_CENTERED_NONE=1 > gpurun_out/r03_c1_ab.log 2>&1 || { tail -20 gpurun_out/r03_c1_ab.log; exit 1; }
cat gpurun_out/r03_c1_ab.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 500 --time-every 100 > gpurun_out/r03_c1_bench.json 2> gpurun_out/r03_c1_bench.err || { tail -20 gpurun_out/r03_c1_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_c1_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
rm -rf gpurun_out/r03_c1_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c1_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 200 --time-every 100 > gpurun_out/r03_c1_prof.log 2>&1 || { tail -20 gpurun_out/r03_c1_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_c1_prof -name run_kernel_stats.csv | head -1)")" > gpurun_out/r03_c1_kstats.txt; cat gpurun_out/r03_c1_kstats.txt
