# r03: Legendre-stage XCD-aware block order A/B (GS_SHT_XCD=0 vs 1) at N_side 256 and 2048
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sht.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_xcd_tests.log 2>&1 || { tail -30 gpurun_out/r03_xcd_tests.log; exit 1; }
tail -1 gpurun_out/r03_xcd_tests.log
for x in 0 1 0 1; do
GS_SHT_XCD=$x timeout -k 10 200 python -u tools/sht_bench.py --nside 256 --lmax 512 --reps 50 > gpurun_out/r03_xcd_256_$x.log 2>&1 || { tail -20 gpurun_out/r03_xcd_256_$x.log; exit 1; }
echo "XCD=$x N256"; grep -v amdgpu gpurun_out/r03_xcd_256_$x.log
done
for x in 0 1; do
GS_SHT_XCD=$x timeout -k 10 300 python -u tools/sht_bench.py --nside 2048 --lmax 4096 --reps 3 > gpurun_out/r03_xcd_2048_$x.log 2>&1 || { tail -20 gpurun_out/r03_xcd_2048_$x.log; exit 1; }
echo "XCD=$x N2048"; grep -v amdgpu gpurun_out/r03_xcd_2048_$x.log
done
