#!/bin/bash
# PMC passes over the VALU Legendre kernels at BASELINE configs[4]'s size
# (tools/sht_bench.py, N_side 2048, l_max 4096): issue / wait counters, the
# scalar-load and LDS counters, then kernel-trace stats.
# usage (GPU box): bash tools/sht_pmc.sh <tag> [nside] [lmax]   -> gpurun_out/shtpmc_<tag>/
set -e
TAG=${1:-r06}
NS=${2:-2048}
LM=${3:-4096}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/shtpmc_$TAG
rm -rf $O; mkdir -p $O
B="tools/sht_bench.py --nside $NS --lmax $LM --reps 2"
K=${KRE:-"k_sht_(anal|synth)_leg"}   # KRE: another kernel regex (the ring stage)
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY \
    SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-include-regex "$K" -d $O/stall -o run \
    --output-format csv -- python3 $B > $O/stall.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-include-regex "$K" -d $O/mem -o run \
    --output-format csv -- python3 $B > $O/mem.log 2>&1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 $B > $O/trace.log 2>&1
echo "sht pmc $TAG done"
