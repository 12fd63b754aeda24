set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r03_b3_$i.json 2> gpurun_out/r03_b3_$i.err || { tail -20 gpurun_out/r03_b3_$i.err; exit 1; }
cat gpurun_out/r03_b3_$i.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --workload centered --nside 256 --lmax 512 --nchains 1 --steps 500 --time-every 100 > gpurun_out/r03_b3_c1.json 2> gpurun_out/r03_b3_c1.err || { tail -20 gpurun_out/r03_b3_c1.err; exit 1; }
cat gpurun_out/r03_b3_c1.json | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
