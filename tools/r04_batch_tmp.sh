set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_sht_mfma.py tests/test_gpu_batched.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_t7.log 2>&1 || { tail -40 gpurun_out/r04_t7.log; exit 1; }
tail -1 gpurun_out/r04_t7.log
O=gpurun_out/r04v; rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/v1 -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma > $O/v1.log 2>&1
grep -E "batch" $O/v1.log
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "mfma" -d $O/pmc -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 3 --mfma > $O/pmc.log 2>&1
GS_SHT_MFA_NT=512 timeout -k 10 100 python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma | grep batch
GS_SHT_MFS_CPW=2 GS_SHT_MFA_CPW=2 timeout -k 10 100 python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma | grep batch
