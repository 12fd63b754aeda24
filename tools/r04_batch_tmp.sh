set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sht_mfma.py tests/test_gpu_batched.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_t8.log 2>&1 || { tail -40 gpurun_out/r04_t8.log; exit 1; }
tail -1 gpurun_out/r04_t8.log
O=gpurun_out/r04ab; rm -rf $O; mkdir -p $O
for rep in 1 2; do
for v in main amap1; do
  if [ $v = main ]; then L=gibbssampler_amd/libgibbs_hip.so; else L=gibbssampler_amd/_exp/lib_$v.so; fi
  GIBBS_HIP_LIB=$PWD/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$rep -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma > $O/${v}_$rep.log 2>&1
  echo "$v $rep $(grep batch $O/${v}_$rep.log)"
done
done
