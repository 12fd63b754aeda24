# r03: Bluestein chirps tabulated at plan time -- SHT / masked tests, SHT 256 timings, masked ASIS trace
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sht.py tests/test_gpu_masked.py tests/test_gpu_baseline_configs.py tests/test_gpu_tt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_chirp_tests.log 2>&1 || { tail -30 gpurun_out/r03_chirp_tests.log; exit 1; }
tail -1 gpurun_out/r03_chirp_tests.log
timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 20 > gpurun_out/r03_chirp_256.log 2>&1 || { tail gpurun_out/r03_chirp_256.log; exit 1; }
grep ncomp gpurun_out/r03_chirp_256.log
timeout -k 10 300 python3 -u bench.py --workload masked_asis --no-cpu-baseline > gpurun_out/r03_chirp_asis.json 2> gpurun_out/r03_chirp_asis.err || { tail -20 gpurun_out/r03_chirp_asis.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_chirp_asis.json')); print('asis', d['value'], d['ms_per_step'])"
rm -rf gpurun_out/r03_chirp_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_chirp_prof -o run --output-format csv -- \
    python3 bench.py --workload masked_asis --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_chirp_prof.log 2>&1 || { tail -20 gpurun_out/r03_chirp_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_chirp_prof -name run_kernel_stats.csv | head -1)")" > gpurun_out/r03_chirp_kstats.txt; grep -i "f2\|leg\|ring" gpurun_out/r03_chirp_kstats.txt
