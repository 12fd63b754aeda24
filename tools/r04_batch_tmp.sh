set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gputest.log 2>&1 || { tail -40 gpurun_out/r04_gputest.log; exit 1; }
tail -1 gpurun_out/r04_gputest.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/r04_default.json 2> gpurun_out/r04_default.err; cut -c1-260 gpurun_out/r04_default.json
O=gpurun_out/r04v; rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/v1 -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma > $O/v1.log 2>&1
grep -E "batch" $O/v1.log
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "mfma" -d $O/pmc -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 3 --mfma > $O/pmc.log 2>&1
