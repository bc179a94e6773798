#!/bin/bash
# Same-box A/B of the tridiagonal reduction: tools/ablib/libgpr_trd_base.so vs the in-tree library,
# alternating, tools/tridiag_probe.py (reduction / syev timings only).  Usage: tools/trd_ab.sh [reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/trd_ab.txt; : > $out
R=${1:-2}
for r in $(seq $R); do
  for v in base new; do
    if [ $v = base ]; then export GPR_HIP_LIB=$PWD/tools/ablib/libgpr_trd_base.so; else unset GPR_HIP_LIB; fi
    echo "== $v" >> $out
    timeout -k 10 200 python -u tools/tridiag_probe.py 512,1100,2048,4096 none 2>/dev/null | grep -E "sytrd|syev" >> $out || exit 1
  done
done
cat $out
