#!/bin/bash
# The headline sweep's issue ceiling, on the GPU box:
#   1. tools/microbench/valu_rate.py: cycles per wave-instruction of every VALU
#      class in the k_cr_sweep<3,0,false,0> loop, 1-8 waves per SIMD
#   2. two PMC passes over the sweep of the default bench (configs[2]):
#      stall / issue counters, and the hardware's VALU class counts
# usage (GPU box): bash tools/issue_probe.sh <tag>   -> gpurun_out/issue_<tag>/
set -e
TAG=${1:-r06}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/issue_$TAG
rm -rf $O; mkdir -p $O
timeout -k 10 240 python3 tools/microbench/valu_rate.py --json $O/valu_rate.json > $O/valu_rate.log 2>&1
echo "valu_rate done"
B="bench.py --no-cpu-baseline --steps 5 --warmup 2 --ramp-ms 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
    SQ_WAVES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex k_cr_sweep -d $O/stall -o run \
    --output-format csv -- python3 $B > $O/stall.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 \
    SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU2 \
    --kernel-include-regex k_cr_sweep -d $O/cls -o run --output-format csv -- python3 $B > $O/cls.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS \
    SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_cr_sweep -d $O/mem -o run \
    --output-format csv -- python3 $B > $O/mem.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 100 --warmup 5 --time-every 100 > $O/trace.log 2>&1
echo "issue probe $TAG done"
