#!/bin/bash
# rocprofv3 kernel stats of tools/sht_bench.py on the GPU box
# usage: bash tools/prof_sht.sh <tag> [nside]
set -e
TAG=${1:-sht}
NS=${2:-512}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 tools/sht_bench.py --nside $NS --reps 5 > gpurun_out/prof_$TAG.log 2>&1
