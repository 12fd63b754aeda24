# r03: mixed small-map SHT shapes (32-l table; T / spin-2 analysis 2 ring groups per lane) -- tests, timings, masked benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py tests/test_gpu_baseline_configs.py tests/test_gpu_tt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_anaseg_tests.log 2>&1 || { tail -30 gpurun_out/r03_anaseg_tests.log; exit 1; }
tail -1 gpurun_out/r03_anaseg_tests.log
timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 20 > gpurun_out/r03_anaseg_256.log 2>&1 || { tail gpurun_out/r03_anaseg_256.log; exit 1; }
grep ncomp gpurun_out/r03_anaseg_256.log
timeout -k 10 120 python3 -u tools/sht_bench.py --nside 64 --lmax 128 --reps 20 > gpurun_out/r03_anaseg_64.log 2>&1 || { tail gpurun_out/r03_anaseg_64.log; exit 1; }
grep ncomp gpurun_out/r03_anaseg_64.log
for w in masked_asis masked_centered_ula; do
timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline > gpurun_out/r03_anaseg_$w.json 2> gpurun_out/r03_anaseg_$w.err || { tail -20 gpurun_out/r03_anaseg_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_anaseg_$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
