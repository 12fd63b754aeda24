set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gputest.log 2>&1 || { tail -30 gpurun_out/r04_gputest.log; exit 1; }
tail -1 gpurun_out/r04_gputest.log
for m in masked_asis masked_noncentered; do
  timeout -k 10 240 python3 bench.py --workload $m --nchains 16 --no-cpu-baseline > gpurun_out/bench_r04_${m}_b16.json 2> gpurun_out/bench_r04_${m}_b16.err
  echo "$m"; cut -c100-250 gpurun_out/bench_r04_${m}_b16.json
done
