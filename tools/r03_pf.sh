# r03: analysis Legendre coefficient prefetch A/B at N_side 2048 (+ SHT tests on the variant)
set -o pipefail
mkdir -p gpurun_out
for v in base a16s16 a16s32 pf16 base; do
  lib=gibbssampler_amd/libgibbs_hip.so; [ $v != base ] && lib=gibbssampler_amd/libgibbs_hip_$v.so
  echo "== $v"
  GIBBS_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u tools/sht_bench.py --nside 2048 --reps 3 > gpurun_out/r03_pf_$v.log 2>&1 || { tail -20 gpurun_out/r03_pf_$v.log; exit 1; }
  grep -i "map2alm\|alm2map" gpurun_out/r03_pf_$v.log | tail -6
done
GIBBS_HIP_LIB=$PWD/gibbssampler_amd/libgibbs_hip_a16s16.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sht.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_pf_tests.log 2>&1 || { tail -20 gpurun_out/r03_pf_tests.log; exit 1; }
tail -1 gpurun_out/r03_pf_tests.log
