# r03: device-resident masked centered loop -- masked tests, HEAD masked bench lines without the CPU leg
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_masked.py tests/test_gpu_surface.py tests/test_gpu_baseline_configs.py tests/test_gpu_tt.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_devloop_tests.log 2>&1 || { tail -30 gpurun_out/r03_devloop_tests.log; exit 1; }
tail -1 gpurun_out/r03_devloop_tests.log
for w in masked_centered_ula masked_centered_ula; do
timeout -k 10 300 python3 -u bench.py --workload $w --no-cpu-baseline > gpurun_out/r03_devloop_$w.json 2> gpurun_out/r03_devloop_$w.err || { tail -20 gpurun_out/r03_devloop_$w.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_devloop_$w.json')); print('$w', d['value'], d['ms_per_step'])"
done
