#!/bin/bash
# PMC passes over the headline sweep of this build (bench.py default, configs[2]):
# stall / issue counters, the hardware's VALU class counts, FETCH_SIZE and
# WRITE_SIZE; then the kernel-trace stats of a 100-step bench.
# usage (GPU box): bash tools/sweep_pmc.sh <tag>   -> gpurun_out/pmc_<tag>/
set -e
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_$TAG
rm -rf $O; mkdir -p $O
B="bench.py --no-cpu-baseline --steps 5 --warmup 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    SQ_WAVES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex k_cr_sweep -d $O/stall -o run \
    --output-format csv -- python3 $B > $O/stall.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
    SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU2 \
    --kernel-include-regex k_cr_sweep -d $O/cls -o run --output-format csv -- python3 $B > $O/cls.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d $O/fetch -o run \
    --output-format csv -- python3 $B > $O/fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d $O/write -o run \
    --output-format csv -- python3 $B > $O/write.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --time-every 100 > $O/trace.log 2>&1
echo "sweep pmc $TAG done"
