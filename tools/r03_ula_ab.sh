# r03: masked_centered_ula A/B -- current library against the 2e3ae4f build (build_variants/lib_prev.so)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in cur prev cur prev; do
    if [ $v = prev ]; then export GIBBS_HIP_LIB=$PWD/build_variants/lib_prev.so; else unset GIBBS_HIP_LIB; fi
    timeout -k 10 300 python3 -u bench.py --workload masked_centered_ula --no-cpu-baseline > gpurun_out/r03_ula_$v.json 2> gpurun_out/r03_ula_$v.err || { tail -20 gpurun_out/r03_ula_$v.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/r03_ula_$v.json')); print('$v', d['value'], d['ms_per_step'])"
done
