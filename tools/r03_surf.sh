# r03: run() graph reuse + pinned-host streaming of the histories; surface bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_surface.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_surf_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_surf_tests.log; exit 1; }
tail -1 gpurun_out/r03_surf_tests.log
for n in 50 500; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline --workload surface_noncentered --steps $n > gpurun_out/r03_surf_$n.json 2> gpurun_out/r03_surf_$n.err || { tail -20 gpurun_out/r03_surf_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_surf_$n.json')); print('surface $n', d['value'], d['ms_per_step'])"
done
