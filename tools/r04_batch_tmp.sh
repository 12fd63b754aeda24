set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04v; rm -rf $O; mkdir -p $O
i=0
for v in "4 4 256 1" "2 4 512 2" "4 2 512 4" "2 2 256 2" "4 4 512 4"; do set -- $v; i=$((i+1))
GS_SHT_RING_NC=$4 GS_SHT_MFS_CPW=$1 GS_SHT_MFA_CPW=$2 GS_SHT_MFA_NT=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/v$i -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --batch 16 --ncomp 2 --reps 10 --mfma > $O/v$i.log 2>&1
echo "v$i $v"; grep batch $O/v$i.log
done
