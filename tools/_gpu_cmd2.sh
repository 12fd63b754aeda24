set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/fdt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fdt -o run -- python3 bench.py --workload centered --nside 256 --lmax 512 --nchains 1 --steps 100 --time-every 1000 --no-cpu-baseline --ramp-ms 0 > gpurun_out/fdt.log 2>&1
f=$(ls gpurun_out/fdt/*/run_kernel_trace.csv gpurun_out/fdt/run_kernel_trace.csv 2>/dev/null | head -1); cp $f gpurun_out/fdt/run_kernel_trace.csv 2>/dev/null || true
python3 tools/ktimeline.py gpurun_out/fdt --skip 200 --n 12
