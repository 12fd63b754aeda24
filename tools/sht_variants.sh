#!/bin/bash
# time tools/sht_bench.py against SHT build variants: bash tools/sht_variants.sh lib1.so lib2.so ...
for lib in "$@"; do
  echo "== $lib"
  GIBBS_HIP_LIB=$lib timeout -k 10 300 python tools/sht_bench.py --nside ${NSIDE:-512} --reps ${REPS:-5} 2>&1 | grep -v amdgpu.ids
done
