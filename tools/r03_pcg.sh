set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gputest2.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_gputest2.log; exit 1; }
tail -2 gpurun_out/r03_gputest2.log
timeout -k 10 300 python -u bench.py --workload masked_centered_pcg --steps 3 --warmup 1 > gpurun_out/r03_bench_pcg.json 2> gpurun_out/r03_bench_pcg.err || { tail -20 gpurun_out/r03_bench_pcg.err; exit 1; }
cat gpurun_out/r03_bench_pcg.json
timeout -k 10 300 python -u bench.py --workload masked_noncentered --steps 3 --warmup 1 > gpurun_out/r03_bench_ncm.json 2> gpurun_out/r03_bench_ncm.err || { tail -20 gpurun_out/r03_bench_ncm.err; exit 1; }
cat gpurun_out/r03_bench_ncm.json
