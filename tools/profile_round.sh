#!/bin/bash
# Round evidence on the GPU box (rocprofv3 + bench lines), all under gpurun_out/:
#   prof_<tag>/trace     kernel trace + stats of the default bench (BASELINE configs[2])
#   prof_<tag>/fetch|write  separate PMC passes (FETCH_SIZE, WRITE_SIZE) of k_cr_sweep
#   bench_<tag>_*.json   bench lines: default (with cpu_baseline), centered C2, asis C4 (per GPU), masked C5
#   prof_<tag>_masked    kernel stats of the masked C5 workload
#   prof_<tag>_sht       kernel stats of tools/sht_bench.py at N_side 2048
# usage (GPU box): bash tools/profile_round.sh <tag>
set -e
TAG=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT" "${OUT}_masked" "${OUT}_sht"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT.trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/fetch" -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/write" -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.write.log" 2>&1
echo "profiles done" 
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err
timeout -k 10 300 python3 bench.py --workload centered --nside 256 --lmax 512 --nchains 1 --no-cpu-baseline \
    > gpurun_out/bench_${TAG}_centered_C2.json 2> gpurun_out/bench_${TAG}_centered_C2.err
timeout -k 10 300 python3 bench.py --workload asis --no-cpu-baseline \
    > gpurun_out/bench_${TAG}_asis_C4.json 2> gpurun_out/bench_${TAG}_asis_C4.err
timeout -k 10 600 python3 bench.py --workload masked > gpurun_out/bench_${TAG}_masked_C5.json \
    2> gpurun_out/bench_${TAG}_masked_C5.err
echo "bench lines done"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "${OUT}_masked" -o run --output-format csv -- \
    python3 bench.py --workload masked --steps 5 --warmup 1 > "${OUT}_masked.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_sht" -o run --output-format csv -- \
    python3 tools/sht_bench.py --nside 2048 --reps 3 > "${OUT}_sht.log" 2>&1
echo "profile $TAG done"
