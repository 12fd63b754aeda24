# r03: kernel stats of the HEAD gibbs_cr + ula line (masked aux CR + MALA, N_side 256 / L 512)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/r03_ula_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_ula_prof -o run --output-format csv -- python3 bench.py --workload masked_centered_ula --steps 40 --warmup 2 --no-cpu-baseline > gpurun_out/r03_ula_prof.log 2>&1 || { tail -20 gpurun_out/r03_ula_prof.log; exit 1; }
tail -1 gpurun_out/r03_ula_prof.log | cut -c1-300
python3 tools/kstats.py "$(dirname "$(find gpurun_out/r03_ula_prof -name run_kernel_stats.csv | head -1)")"
