#!/bin/bash
# Profile the default bench command on the GPU box (rocprofv3): kernel trace +
# stats, then separate PMC passes for FETCH_SIZE and WRITE_SIZE of the sweep.
# usage (GPU box): bash tools/profile_round.sh <tag>
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT.trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/fetch" -o run \
    --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/write" -o run \
    --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.write.log" 2>&1
echo "profile $TAG done"
