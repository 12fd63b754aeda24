# r03: GPU suite + bench lines of the harmonic configs (default no-store and stored variants)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_ba_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_ba_tests.log; exit 1; }
tail -1 gpurun_out/r03_ba_tests.log
run() { timeout -k 10 400 python -u bench.py "$@" > gpurun_out/r03_ba_$TAG.json 2> gpurun_out/r03_ba_$TAG.err || { tail -20 gpurun_out/r03_ba_$TAG.err; exit 1; }; python3 -c "import json; d=json.load(open('gpurun_out/r03_ba_$TAG.json')); r=d['roofline']; print('$TAG', d['value'], d['ms_per_step'], r['bound'], r['frac'], r['avg_launch_ms'])"; }
TAG=default; run
TAG=store; run --no-cpu-baseline --skymap store
TAG=c2; run --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 500 --time-every 100
TAG=c2store; run --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 500 --time-every 100 --skymap store
TAG=c4; run --no-cpu-baseline --workload asis
TAG=surface; run --no-cpu-baseline --workload surface_noncentered
GS_AB_NOSTORE=1 timeout -k 10 300 python -u tools/step_ab.py noncentered 1024 512 32 50 GS_SWEEP_TW=2 GS_SWEEP_TW=1 GS_SWEEP_TW=4 > gpurun_out/r03_ba_twab.log 2>&1 || { tail -20 gpurun_out/r03_ba_twab.log; exit 1; }
cat gpurun_out/r03_ba_twab.log
timeout -k 10 120 python -u tools/prologue_probe.py > gpurun_out/r03_prologue.log 2>&1 || { tail -20 gpurun_out/r03_prologue.log; exit 1; }; cat gpurun_out/r03_prologue.log
