# r03 final-tree check: whole -m gpu suite, smoke(), default bench line, HEAD gibbs_cr + ula line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_final_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_final_tests.log; exit 1; }
tail -2 gpurun_out/r03_final_tests.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final_smoke.txt 2>&1 || { tail -20 gpurun_out/r03_final_smoke.txt; exit 1; }
cat gpurun_out/r03_final_smoke.txt
timeout -k 10 300 python -u bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err || { tail -20 gpurun_out/r03_final_bench.err; exit 1; }
cat gpurun_out/r03_final_bench.json
timeout -k 10 300 python -u bench.py --workload masked_centered_ula --no-cpu-baseline > gpurun_out/r03_final_ula.json 2> gpurun_out/r03_final_ula.err || { tail -20 gpurun_out/r03_final_ula.err; exit 1; }
cat gpurun_out/r03_final_ula.json
