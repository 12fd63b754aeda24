#!/bin/bash
# Round evidence on the GPU box (rocprofv3 + bench lines), all under gpurun_out/:
#   prof_<tag>/trace        kernel trace + stats of the default bench (BASELINE configs[2])
#   prof_<tag>/fetch|write  separate PMC passes (FETCH_SIZE, WRITE_SIZE) of k_cr_sweep
#   prof_<tag>/valu         PMC pass: SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE
#   bench_<tag>_*.json      bench lines: default (with cpu_baseline), centered C2, asis C4 (per GPU),
#                           masked C5, HEAD's masked modes (masked_asis, masked_centered_ula)
#   prof_<tag>_<mode>       kernel stats of the masked workloads, SHT at N_side 2048
# usage (GPU box): bash tools/profile_round.sh <tag>
set -e
TAG=${1:-r02}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
rm -rf "$OUT" "${OUT}_masked" "${OUT}_sht" "${OUT}_masked_asis" "${OUT}_masked_ula" "${OUT}_c2"
B="python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --time-every 20"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- $B > "$OUT.trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/fetch" -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/write" -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
    --kernel-include-regex k_cr_sweep -d "$OUT/valu" -o run \
    --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT.valu.log" 2>&1
echo "profiles done"
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err
timeout -k 10 300 python3 bench.py --workload centered --nside 256 --lmax 512 --nchains 1 --steps 500 --time-every 100 \
    > gpurun_out/bench_${TAG}_centered_C2.json 2> gpurun_out/bench_${TAG}_centered_C2.err
timeout -k 10 300 python3 bench.py --workload asis --time-every 10 \
    > gpurun_out/bench_${TAG}_asis_C4.json 2> gpurun_out/bench_${TAG}_asis_C4.err
timeout -k 10 600 python3 bench.py --workload masked > gpurun_out/bench_${TAG}_masked_C5.json \
    2> gpurun_out/bench_${TAG}_masked_C5.err
timeout -k 10 300 python3 bench.py --workload masked_asis > gpurun_out/bench_${TAG}_masked_asis.json \
    2> gpurun_out/bench_${TAG}_masked_asis.err
timeout -k 10 300 python3 bench.py --workload masked_centered_ula > gpurun_out/bench_${TAG}_masked_ula.json \
    2> gpurun_out/bench_${TAG}_masked_ula.err
timeout -k 10 400 python3 bench.py --no-cpu-baseline --skymap none > gpurun_out/bench_${TAG}_default_nostore.json \
    2> gpurun_out/bench_${TAG}_default_nostore.err
echo "bench lines done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_c2" -o run --output-format csv -- \
    python3 bench.py --workload centered --nside 256 --lmax 512 --nchains 1 --steps 200 --time-every 100 > "${OUT}_c2.log" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "${OUT}_masked" -o run --output-format csv -- \
    python3 bench.py --workload masked --steps 5 --warmup 1 > "${OUT}_masked.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_masked_asis" -o run --output-format csv -- \
    python3 bench.py --workload masked_asis --steps 3 --warmup 1 > "${OUT}_masked_asis.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_sht" -o run --output-format csv -- \
    python3 tools/sht_bench.py --nside 2048 --reps 3 > "${OUT}_sht.log" 2>&1
echo "profile $TAG done"
