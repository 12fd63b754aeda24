#!/bin/bash
# One GPU-box session: the -m gpu suite, then optional extra steps (tools/*.sh
# parts), stopping at the first GPU fault / abort / time limit (exit 124, 134,
# 137, 139); an ordinary test failure (exit 1) lets the later steps run.
# usage (GPU box): bash tools/gpu_session.sh <tag> [command ...]
TAG=${1:-r06}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gputest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "gpu suite ended with $rc: stopping"; exit $rc; fi
for c in "$@"; do
    echo "== $c"
    bash -c "$c"
    r=$?
    if [ $r -ne 0 ]; then echo "step ended with $r: stopping"; exit $r; fi
done
exit $rc
