#!/bin/bash
# time the sweep for several rows-per-task settings (run on the GPU box)
for r in 64 32 16 8 4; do
  echo "rows=$r"; GS_SWEEP_ROWS=$r timeout -k 10 120 python tools/sweep_variants.py build/variants/lib_CUR.so | tail -1 || exit 1
done
