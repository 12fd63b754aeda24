# r03: f2 Gram pass on the fp64 MFMA -- masked / scale tests, masked ASIS A/B (MFMA vs VALU Gram), kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_masked.py tests/test_gpu_scale.py tests/test_gpu_baseline_configs.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gram_tests.log 2>&1 || { tail -30 gpurun_out/r03_gram_tests.log; exit 1; }
tail -1 gpurun_out/r03_gram_tests.log
for v in mfma valu mfma valu; do
    if [ $v = valu ]; then export GS_F2_GRAM_VALU=1; else unset GS_F2_GRAM_VALU; fi
    timeout -k 10 300 python3 -u bench.py --workload masked_asis --no-cpu-baseline > gpurun_out/r03_gram_asis_$v.json 2> gpurun_out/r03_gram_asis_$v.err || { tail -20 gpurun_out/r03_gram_asis_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03_gram_asis_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
unset GS_F2_GRAM_VALU
rm -rf gpurun_out/r03_gram_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_gram_prof -o run --output-format csv -- \
    python3 bench.py --workload masked_asis --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r03_gram_prof.log 2>&1 || { tail -20 gpurun_out/r03_gram_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_gram_prof -name run_kernel_stats.csv | head -1)")" > gpurun_out/r03_gram_kstats.txt; grep -i "f2\|leg\|ring" gpurun_out/r03_gram_kstats.txt
