# round-3 state check: the whole -m gpu suite, the default bench line, configs[1]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_verify_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_verify_tests.log; exit 1; }
tail -2 gpurun_out/r03_verify_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/r03_verify_bench.json 2> gpurun_out/r03_verify_bench.err || { tail -20 gpurun_out/r03_verify_bench.err; exit 1; }
cat gpurun_out/r03_verify_bench.json
timeout -k 10 300 python -u bench.py --workload centered > gpurun_out/r03_verify_c2.json 2> gpurun_out/r03_verify_c2.err || { tail -20 gpurun_out/r03_verify_c2.err; exit 1; }
cat gpurun_out/r03_verify_c2.json
