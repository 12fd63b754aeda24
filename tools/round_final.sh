# Round-end evidence on the GPU box: the -m gpu suite, smoke(), the default
# bench line (with its CPU baseline) and profile_round.sh part d (HEAD's masked
# modes at 16 chains per GPU + the PCG kernel stats), all under gpurun_out/.
# usage: bash tools/round_final.sh <tag>
set -e
TAG=${1:-r05}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_final_gputest.log 2>&1 || { tail -40 gpurun_out/${TAG}_final_gputest.log; exit 1; }
tail -1 gpurun_out/${TAG}_final_gputest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_final_smoke.txt 2>&1 && echo smoke ok
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_final_bench.json 2> gpurun_out/${TAG}_final_bench.err; cut -c1-200 gpurun_out/${TAG}_final_bench.json
bash tools/profile_round.sh $TAG d
bash tools/profile_round.sh $TAG e
for m in masked_asis masked_centered_ula masked_centered_pcg masked_noncentered; do echo "$m $(cut -c90-190 gpurun_out/bench_${TAG}_${m}_b16.json)"; echo "$m galactic $(cut -c90-190 gpurun_out/bench_${TAG}_${m}_b16_galactic.json)"; done
