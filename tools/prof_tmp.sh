set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for w in masked_centered_pcg masked_centered_ula masked_asis; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pf_$w -o run -- python3 bench.py --workload $w --nchains 16 --steps 2 --warmup 1 > gpurun_out/pf_$w.json 2>gpurun_out/pf_$w.err
done
ls -R gpurun_out | head -40
