# r03: ring stage (inlined FFTs, LDS twiddles, 32-bit phase reduction) -- SHT / masked tests,
# N_side 256 timings, N_side 2048 analysis prefetch-distance variants, masked ASIS bench
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_ring_tests.log 2>&1 || { tail -30 gpurun_out/r03_ring_tests.log; exit 1; }
tail -1 gpurun_out/r03_ring_tests.log
timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 20 > gpurun_out/r03_ring_256.log 2>&1 || { tail gpurun_out/r03_ring_256.log; exit 1; }
cat gpurun_out/r03_ring_256.log
for v in default pf0 pf8 pf24 pf32; do
    if [ $v = default ]; then lib=gibbssampler_amd/libgibbs_hip.so; else lib=build_variants/lib_$v.so; fi
    echo "== $v"
    GIBBS_HIP_LIB=$PWD/$lib timeout -k 10 200 python3 -u tools/sht_bench.py --nside 2048 --reps 3 > gpurun_out/r03_ring_2048_$v.log 2>&1 || { tail gpurun_out/r03_ring_2048_$v.log; exit 1; }
    grep ncomp=3 gpurun_out/r03_ring_2048_$v.log
done
timeout -k 10 300 python3 -u bench.py --workload masked_asis > gpurun_out/r03_ring_masked_asis.json 2> gpurun_out/r03_ring_masked_asis.err || { tail -20 gpurun_out/r03_ring_masked_asis.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_ring_masked_asis.json')); print(d['value'], d['ms_per_step'])"
