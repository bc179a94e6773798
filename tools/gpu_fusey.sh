#!/bin/bash
# gpr_fit with y solved inside the factorisation (GPR_FUSE_Y) on C5 (its fit) and C1-style fits
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/fusey.txt; : > $out
for r in 1 2; do
  for v in 0 1; do
    GPR_FUSE_Y=$v timeout -k 10 200 python bench_split.py > gpurun_out/fy.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/fy.json'));print('fuse_y=$v C5', round(d['ms_per_step'],1))" >> $out
  done
done
