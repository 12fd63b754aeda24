# round-3 masked measurements: the new SHT test, HEAD's masked modes and configs[4] with their CPU legs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sht.py -x -q -k cpu_baseline --timeout 200 --timeout-method thread > gpurun_out/r03_sht_cpu_test.log 2>&1 || { tail -30 gpurun_out/r03_sht_cpu_test.log; exit 1; }
tail -1 gpurun_out/r03_sht_cpu_test.log
for w in masked_centered_ula masked_centered_pcg masked_asis masked_noncentered; do
  timeout -k 10 600 python -u bench.py --workload $w --steps 3 --warmup 1 > gpurun_out/r03_bench_$w.json 2> gpurun_out/r03_bench_$w.err || { tail -20 gpurun_out/r03_bench_$w.err; exit 1; }
  cat gpurun_out/r03_bench_$w.json
done
timeout -k 10 900 python -u bench.py --workload masked --steps 5 --warmup 1 > gpurun_out/r03_bench_masked_C5.json 2> gpurun_out/r03_bench_masked_C5.err || { tail -20 gpurun_out/r03_bench_masked_C5.err; exit 1; }
cat gpurun_out/r03_bench_masked_C5.json
