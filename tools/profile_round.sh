#!/bin/bash
# Round evidence on the GPU box (rocprofv3 + bench lines), all under gpurun_out/:
#   prof_<tag>/trace          kernel trace + stats of the default bench (BASELINE configs[2])
#   prof_<tag>/<v>/fetch|write|valu   separate PMC passes over k_cr_sweep for each bench variant <v>:
#                             default (no-store), store, c2 (configs[1] shape), c4 (asis per GPU);
#                             FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
#   bench_<tag>_*.json        bench lines: default (with cpu_baseline), stored sky map, centered C2,
#                             asis C4 (per GPU), the drop-in surface, masked C5, HEAD's masked modes
#   prof_<tag>_<mode>         kernel stats of configs[1], the masked workloads, SHT at N_side 2048
# usage (GPU box): bash tools/profile_round.sh <tag> [a|b|all]   (then python tools/summarize_profile.py <tag>)
#   a: the harmonic trace, PMC passes and harmonic bench lines; b: the masked bench lines and the
#   masked / configs[1] / SHT kernel stats (two gpurun calls stay within one call's time limit)
set -e
TAG=${1:-r03}
PART=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
if [ "$PART" != b ]; then
rm -rf "$OUT"
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
    python3 bench.py --steps 100 --warmup 5 --no-cpu-baseline --time-every 100 > "$OUT.trace.log" 2>&1
pmc() {  # <variant> <bench args...>
    local v=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/$v/fetch" -o run \
        --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT.$v.fetch.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/$v/write" -o run \
        --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT.$v.write.log" 2>&1
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
        --kernel-include-regex k_cr_sweep -d "$OUT/$v/valu" -o run \
        --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$OUT.$v.valu.log" 2>&1
}
pmc default --steps 5 --warmup 2
pmc store --steps 5 --warmup 2 --skymap store
pmc c2 --workload centered --nside 256 --lmax 512 --nchains 1 --steps 20 --warmup 2 --time-every 100
pmc c4 --workload asis --steps 5 --warmup 2
echo "profiles done"
timeout -k 10 400 python3 bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err
timeout -k 10 400 python3 bench.py --no-cpu-baseline --skymap store > gpurun_out/bench_${TAG}_default_store.json \
    2> gpurun_out/bench_${TAG}_default_store.err
timeout -k 10 300 python3 bench.py --workload centered --nside 256 --lmax 512 --nchains 1 --time-every 100 \
    > gpurun_out/bench_${TAG}_centered_C2.json 2> gpurun_out/bench_${TAG}_centered_C2.err
timeout -k 10 300 python3 bench.py --workload asis \
    > gpurun_out/bench_${TAG}_asis_C4.json 2> gpurun_out/bench_${TAG}_asis_C4.err
timeout -k 10 300 python3 bench.py --workload surface_noncentered --no-cpu-baseline \
    > gpurun_out/bench_${TAG}_surface_C3.json 2> gpurun_out/bench_${TAG}_surface_C3.err
fi
if [ "$PART" != a ]; then
rm -rf "${OUT}_masked" "${OUT}_sht" "${OUT}_masked_asis" "${OUT}_c2"
timeout -k 10 600 python3 bench.py --workload masked > gpurun_out/bench_${TAG}_masked_C5.json \
    2> gpurun_out/bench_${TAG}_masked_C5.err
for m in masked_asis masked_centered_ula masked_centered_pcg masked_noncentered; do
    timeout -k 10 300 python3 bench.py --workload $m > gpurun_out/bench_${TAG}_$m.json 2> gpurun_out/bench_${TAG}_$m.err
done
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
fi
