# r03: segmented SHT launch changes (analysis early exit; synthesis split by m range) -- interleaved A/B of sht_bench at N_side 256
# (base = the tree before the change, GIBBS_HIP_LIB), the SHT tests, then the PCG line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/r03_synsplit.log
for k in 1 2 3; do
  echo "== base $k" >> gpurun_out/r03_synsplit.log
  GIBBS_HIP_LIB=$PWD/gibbssampler_amd/libgibbs_hip_base.so timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 50 >> gpurun_out/r03_synsplit.log 2>&1 || exit 1
  echo "== new $k" >> gpurun_out/r03_synsplit.log
  timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 50 >> gpurun_out/r03_synsplit.log 2>&1 || exit 1
done
grep -E "==|ncomp=2" gpurun_out/r03_synsplit.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_synsplit_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_synsplit_tests.log; exit 1; }
tail -1 gpurun_out/r03_synsplit_tests.log
