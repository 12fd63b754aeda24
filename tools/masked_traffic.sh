#!/bin/bash
# HBM traffic of ONE bench step of every masked line:
# FETCH_SIZE / WRITE_SIZE passes over tools/step_traffic.py (all kernels; the
# step's dispatches sit between two marker launches).
# usage (GPU box): bash tools/masked_traffic.sh <tag> [workload:nchains:mask[:nside:lmax] ...]
set -e
TAG=${1:-r06}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/traffic_$TAG
mkdir -p $O
for spec in "$@"; do
    IFS=: read w nch mask ns lm <<< "$spec"
    extra=""
    [ -n "$ns" ] && extra="--nside $ns --lmax $lm"
    d=$O/${w}_b${nch}_${mask}${ns:+_n$ns}
    rm -rf $d; mkdir -p $d
    for c in FETCH_SIZE WRITE_SIZE; do
        lc=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
        timeout -s KILL 300 rocprofv3 --pmc $c -d $d/$lc -o run --output-format csv -- \
            python3 tools/step_traffic.py --workload $w --nchains $nch --mask $mask $extra > $d/$lc.log 2>&1
    done
    echo "traffic $w $nch $mask done"
done
