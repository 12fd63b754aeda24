# r03 final state check: the whole -m gpu suite, smoke(), the default bench line, the ULA line again
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_final_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_final_tests.log; exit 1; }
tail -2 gpurun_out/r03_final_tests.log
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03_final_smoke.log 2>&1 || { tail -20 gpurun_out/r03_final_smoke.log; exit 1; }
tail -1 gpurun_out/r03_final_smoke.log
timeout -k 10 300 python3 -u bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err || { tail -20 gpurun_out/r03_final_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_final_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 -u bench.py --workload masked_centered_ula > gpurun_out/r03_final_ula.json 2> gpurun_out/r03_final_ula.err || { tail -20 gpurun_out/r03_final_ula.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_final_ula.json')); print('ula', d['value'], d['ms_per_step'])"
