# r03: full GPU suite twice with the C_l pre-draw on (GC paused during captures)
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03_diag2_$k.log 2>&1 || { grep -n "PASSED\|FAILED\|ERROR" gpurun_out/r03_diag2_$k.log | tail -3; tail -5 gpurun_out/r03_diag2_$k.log; exit 1; }
tail -1 gpurun_out/r03_diag2_$k.log
done
GS_AB_NOSTORE=1 timeout -k 10 300 python3 -u tools/step_ab.py centered 512 256 1 500 GS_CLS_PRE=0 GS_CLS_PRE=1 > gpurun_out/r03_clspre_ab.log 2>&1 || { tail -20 gpurun_out/r03_clspre_ab.log; exit 1; }
cat gpurun_out/r03_clspre_ab.log
