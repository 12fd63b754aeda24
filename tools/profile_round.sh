#!/bin/bash
# Round evidence on the GPU box (rocprofv3 + bench lines), all under gpurun_out/:
#   prof_<tag>/trace          kernel trace + stats of the default bench (BASELINE configs[2])
#   prof_<tag>/<v>/fetch|write|valu   separate PMC passes over k_cr_sweep for each bench variant <v>:
#                             default (no-store), store, c2 (configs[1] shape), c4 (asis per GPU);
#                             FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
#   bench_<tag>_*.json        bench lines: default (with cpu_baseline), stored sky map, centered C2,
#                             asis C4 (per GPU), the drop-in surface, masked C5, HEAD's masked modes
#   prof_<tag>_<mode>         kernel stats of configs[1], the masked workloads, SHT at N_side 2048
# usage (GPU box): bash tools/profile_round.sh <tag> [a|b|c|d|all]   (then python tools/summarize_profile.py <tag>)
#   a: the harmonic trace, PMC passes and harmonic bench lines (= p then h); b: the masked bench lines and the
#   masked / configs[1] / SHT kernel stats (two gpurun calls stay within one call's time limit);
#   c (r04): the chain-batched SHT (N_side 256, 16 spin-2 maps, matrix-core Legendre tables) --
#   kernel stats and FETCH_SIZE / WRITE_SIZE / SQ passes -- and the N_side 2048 recurrence kernels'
#   PMC passes; d (r04): HEAD's masked modes at 16 chains per GPU (bench lines + kernel stats);
#   e (r05): the same on the galactic-like mask (--mask galactic) + the ASIS kernel stats
#   (python tools/summarize_sht_pmc.py <tag> folds c's passes into profiles/pmc_traffic.json)
set -e
TAG=${1:-r03}
PART=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/prof_$TAG
if [ "$PART" = a ] || [ "$PART" = p ] || [ "$PART" = all ]; then
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
fi
# h: the harmonic bench lines alone (after summarize_profile.py has folded part p's passes into
# profiles/pmc_traffic.json, so the lines' roofline reads this build's counters)
if [ "$PART" = a ] || [ "$PART" = h ] || [ "$PART" = all ]; then
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
if [ "$PART" = c ]; then
O=gpurun_out/prof_${TAG}_shtb; rm -rf $O; mkdir -p $O
A="tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 5 --mfma"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $A > $O/trace.log 2>&1
for pass in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-include-regex "k_sht" -d $O/$n -o run --output-format csv \
        -- python3 $A > $O/$n.log 2>&1
done
# the fused PCG operator's ring stage (tools/sht_bench.py --apply: band-masked weights)
O=gpurun_out/prof_${TAG}_shta; rm -rf $O; mkdir -p $O
A="tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 5 --mfma --apply"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $A > $O/trace.log 2>&1
for pass in "FETCH_SIZE" "WRITE_SIZE" \
    "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 60 rocprofv3 --pmc $pass --kernel-include-regex "k_sht_apply_ring|k_pair_support" -d $O/$n -o run \
        --output-format csv -- python3 $A > $O/$n.log 2>&1
done
O=gpurun_out/prof_${TAG}_sht2048; rm -rf $O; mkdir -p $O
A="tools/sht_bench.py --nside 2048 --reps 2"
for pass in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
    n=$(echo $pass | cut -d' ' -f1 | tr 'A-Z' 'a-z')
    timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex "k_sht_(anal|synth)_leg" -d $O/$n -o run \
        --output-format csv -- python3 $A > $O/$n.log 2>&1
done
echo "profile $TAG c done"
exit 0
fi
if [ "$PART" = d ]; then
for m in masked_asis masked_centered_ula masked_centered_pcg masked_noncentered; do
    timeout -k 10 300 python3 bench.py --workload $m --nchains 16 > gpurun_out/bench_${TAG}_${m}_b16.json \
        2> gpurun_out/bench_${TAG}_${m}_b16.err
done
rm -rf "${OUT}_pcg_b16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_pcg_b16" -o run --output-format csv -- \
    python3 bench.py --workload masked_centered_pcg --nchains 16 --steps 2 --warmup 1 --no-cpu-baseline \
    > "${OUT}_pcg_b16.log" 2>&1
echo "profile $TAG d done"
exit 0
fi
if [ "$PART" = e ]; then
# r05: HEAD's masked modes at 16 chains per GPU on the galactic-like mask (the
# band mask's lines are part d), and the ASIS kernel stats
for m in masked_asis masked_centered_ula masked_centered_pcg masked_noncentered; do
    timeout -k 10 300 python3 bench.py --workload $m --nchains 16 --mask galactic --no-cpu-baseline \
        > gpurun_out/bench_${TAG}_${m}_b16_galactic.json 2> gpurun_out/bench_${TAG}_${m}_b16_galactic.err
done
rm -rf "${OUT}_asis_b16"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "${OUT}_asis_b16" -o run --output-format csv -- \
    python3 bench.py --workload masked_asis --nchains 16 --steps 2 --warmup 1 --no-cpu-baseline \
    > "${OUT}_asis_b16.log" 2>&1
echo "profile $TAG e done"
exit 0
fi
if [ "$PART" = b ] || [ "$PART" = all ]; then
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
