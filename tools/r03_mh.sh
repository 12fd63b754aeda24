# r03: MH kernel A/B (k_mh_reg vs k_mh_fused) at configs[2], kernel stats, tests
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_mh_tests.log 2>&1 || { echo TESTS FAILED; tail -30 gpurun_out/r03_mh_tests.log; exit 1; }
tail -2 gpurun_out/r03_mh_tests.log
timeout -k 10 300 python -u tools/step_ab.py noncentered 1024 512 32 50 GS_MH_FUSED=1 GS_MH_NONE=1 > gpurun_out/r03_mh_ab.log 2>&1 || { tail -20 gpurun_out/r03_mh_ab.log; exit 1; }
cat gpurun_out/r03_mh_ab.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r03_mh_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_mh_prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-every 20 > gpurun_out/r03_mh_prof.log 2>&1 || { tail -20 gpurun_out/r03_mh_prof.log; exit 1; }
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_mh_prof -name run_kernel_stats.csv | head -1)")"
GIBBS_HIP_LIB=gibbssampler_amd/libgibbs_hip_timeline.so timeout -k 10 200 python -u tools/mh_timeline.py > gpurun_out/r03_tl.log 2>&1 || { tail -20 gpurun_out/r03_tl.log; exit 1; }
cat gpurun_out/r03_tl.log
