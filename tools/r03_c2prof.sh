# r03: configs[1] bench line + kernel stats after the variates change
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --time-every 100 > gpurun_out/r03_c2b.json 2> gpurun_out/r03_c2b.err || { tail -20 gpurun_out/r03_c2b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_c2b.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c2prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 200 --time-every 100 > gpurun_out/r03_c2prof.log 2>&1 || { tail -20 gpurun_out/r03_c2prof.log; exit 1; }
python3 tools/kstats.py gpurun_out/r03_c2prof > gpurun_out/r03_c2prof_k.txt && head -8 gpurun_out/r03_c2prof_k.txt
