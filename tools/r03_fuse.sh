# r03: fused beam / N^-1 weight into the SHT input loads + CG alpha folded into the update:
# whole -m gpu suite, then the HEAD masked lines (PCG, ULA, ASIS) and a kernel-stats pass of the PCG line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_fuse_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_fuse_tests.log; exit 1; }
tail -2 gpurun_out/r03_fuse_tests.log
for w in masked_centered_pcg masked_centered_ula masked_asis; do
timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline > gpurun_out/r03_fuse_$w.json 2> gpurun_out/r03_fuse_$w.err || { tail -20 gpurun_out/r03_fuse_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_fuse_$w.json')); print('$w', d['value'], d['ms_per_step'], d.get('pcg'))"
done
rm -rf gpurun_out/r03_fuse_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_fuse_prof -o run --output-format csv -- python3 bench.py --workload masked_centered_pcg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03_fuse_prof.log 2>&1 || { tail -20 gpurun_out/r03_fuse_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_fuse_prof -name run_kernel_stats.csv | head -1)")"
