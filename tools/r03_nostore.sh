# r03: the no-store sweep (--skymap none): bench lines (both variants, interleaved) + PMC passes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in none store none store; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --skymap $v > gpurun_out/r03_ns_$v.json 2> gpurun_out/r03_ns_$v.err || { tail -20 gpurun_out/r03_ns_$v.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03_ns_$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
done
OUT=gpurun_out/prof_r03ns
rm -rf $OUT
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --skymap none > $OUT.fetch.log 2>&1 || { tail -5 $OUT.fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_cr_sweep -d "$OUT/write" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --skymap none > $OUT.write.log 2>&1 || { tail -5 $OUT.write.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-include-regex k_cr_sweep -d "$OUT/valu" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --skymap none > $OUT.valu.log 2>&1 || { tail -5 $OUT.valu.log; exit 1; }
find $OUT -name "*counter_collection.csv" | head -5
