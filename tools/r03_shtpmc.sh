# r03: stall breakdown of the N_side 2048 Legendre kernels (one PMC pass)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE \
    --kernel-include-regex "k_sht_(anal|synth)_leg" -d gpurun_out/r03_shtpmc -o run --output-format csv -- \
    python3 tools/sht_bench.py --nside 2048 --reps 1 > gpurun_out/r03_shtpmc.log 2>&1 || { tail -20 gpurun_out/r03_shtpmc.log; exit 1; }
echo done
