# r03: default bench at longer timed regions (steady clocks)
set -o pipefail
mkdir -p gpurun_out
for n in 50 500 2000; do
timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps $n > gpurun_out/r03_steps_$n.json 2> gpurun_out/r03_steps_$n.err || { tail -20 gpurun_out/r03_steps_$n.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_steps_$n.json')); r=d['roofline']; print('default $n', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], d['config'].get('time_every'))"
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline --workload surface_noncentered --steps 2000 > gpurun_out/r03_steps_s2000.json 2> gpurun_out/r03_steps_s2000.err || { tail -20 gpurun_out/r03_steps_s2000.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_steps_s2000.json')); print('surface 2000', d['value'], d['ms_per_step'])"
