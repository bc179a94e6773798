#!/bin/bash
# Same-box A/B of the batched quadrature: tools/ablib/libgpr_trd_base.so vs the in-tree library,
# alternating (tools/quad_batched_probe.py at a few sizes).  Usage: tools/quad_ab.sh [reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/quad_ab.txt; : > $out
for r in $(seq ${1:-2}); do
  for v in base new; do
    if [ $v = base ]; then export GPR_HIP_LIB=$PWD/tools/ablib/libgpr_trd_base.so; else unset GPR_HIP_LIB; fi
    for sz in "4096 128" "4096 200" "2048 128" "1100 100"; do
      echo -n "$v " >> $out
      timeout -k 10 120 python -u tools/quad_batched_probe.py $sz 2>/dev/null | tail -1 >> $out || exit 1
    done
  done
done
cat $out
