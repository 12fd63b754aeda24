set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
rm -rf gpurun_out/r03_ldspmc
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --kernel-include-regex "ring|leg" -d gpurun_out/r03_ldspmc -o run --output-format csv -- python3 tools/sht_bench.py --nside 256 --reps 2 > gpurun_out/r03_ldspmc.log 2>&1 || { tail -5 gpurun_out/r03_ldspmc.log; exit 1; }
f=$(find gpurun_out/r03_ldspmc -name "run_counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'][:60]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    n[(k, r['Counter_Name'])] += 1
for k, d in acc.items():
    print(k, {c: round(v / n[(k, c)]) for c, v in d.items()})
PY
