# r03 final-tree check after the analysis early exit: whole -m gpu suite, smoke(), default bench line, configs[1], configs[4]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_final3_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_final3_tests.log; exit 1; }
tail -2 gpurun_out/r03_final3_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final3_smoke.txt 2>&1 || { tail -20 gpurun_out/r03_final3_smoke.txt; exit 1; }
cat gpurun_out/r03_final3_smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r03_final3_bench.json 2> gpurun_out/r03_final3_bench.err || { tail -20 gpurun_out/r03_final3_bench.err; exit 1; }
cut -c1-400 gpurun_out/r03_final3_bench.json
timeout -k 10 300 python -u bench.py --workload centered --no-cpu-baseline > gpurun_out/r03_final3_c2.json 2> gpurun_out/r03_final3_c2.err || { tail -20 gpurun_out/r03_final3_c2.err; exit 1; }
cut -c1-300 gpurun_out/r03_final3_c2.json
timeout -k 10 400 python -u bench.py --workload masked --no-cpu-baseline > gpurun_out/r03_final3_c5.json 2> gpurun_out/r03_final3_c5.err || { tail -20 gpurun_out/r03_final3_c5.err; exit 1; }
cut -c1-300 gpurun_out/r03_final3_c5.json
