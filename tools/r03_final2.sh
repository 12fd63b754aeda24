# r03 final tree: the whole -m gpu suite, smoke(), the default line, and the masked lines the device-resident runners changed
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_final2_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_final2_tests.log; exit 1; }
tail -2 gpurun_out/r03_final2_tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_final2_smoke.log 2>&1 || { tail -20 gpurun_out/r03_final2_smoke.log; exit 1; }
tail -1 gpurun_out/r03_final2_smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_final2_bench.json 2> gpurun_out/r03_final2_bench.err || { tail -20 gpurun_out/r03_final2_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_final2_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
for w in masked_centered_ula masked; do
timeout -k 10 600 python3 -u bench.py --workload $w > gpurun_out/bench_r03_$w.json 2> gpurun_out/bench_r03_$w.err || { tail -20 gpurun_out/bench_r03_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03_$w.json')); print('$w', d['value'], d['ms_per_step'], (d.get('cpu_baseline') or {}).get('value'))"
done
