set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r04_default.json 2> gpurun_out/r04_default.err; cut -c100-200 gpurun_out/r04_default.json
O=gpurun_out/r04ab; rm -rf $O; mkdir -p $O
for rep in 1 2; do
for v in main nopad noxcd none; do
  if [ $v = main ]; then L=gibbssampler_amd/libgibbs_hip.so; else L=gibbssampler_amd/_exp/lib_$v.so; fi
  GIBBS_HIP_LIB=$PWD/$L timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/${v}_$rep -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma > $O/${v}_$rep.log 2>&1
  echo "$v $rep $(grep batch $O/${v}_$rep.log)"
done
done
