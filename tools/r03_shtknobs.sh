# r03: small-map SHT (N_side 256 / L 512, HEAD's masked modes) -- plan knobs scan + kernel stats
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # <tag> <env...>
    local tag=$1; shift
    echo "== $tag" >> gpurun_out/r03_shtknobs.log
    env "$@" timeout -k 10 120 python3 -u tools/sht_bench.py --nside 256 --reps 20 >> gpurun_out/r03_shtknobs.log 2>&1
}
: > gpurun_out/r03_shtknobs.log
run default A=1 || exit 1
run seg32 GS_SHT_SEG=32 || exit 1
run seg128 GS_SHT_SEG=128 || exit 1
run ana2_seg32 GS_SHT_ANA=2,0 GS_SHT_SEG=32 || exit 1
run ana2_seg16 GS_SHT_ANA=2,0 GS_SHT_SEG=16 || exit 1
run ana4_seg16 GS_SHT_ANA=4,0 GS_SHT_SEG=16 || exit 1
run nomerge GS_SHT_MERGE_RINGS=0 || exit 1
cat gpurun_out/r03_shtknobs.log
rm -rf gpurun_out/r03_sht256_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_sht256_prof -o run --output-format csv -- \
    python3 tools/sht_bench.py --nside 256 --reps 20 > gpurun_out/r03_sht256_prof.log 2>&1 || exit 1
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_sht256_prof -name run_kernel_stats.csv | head -1)")"
