#!/bin/bash
# Same-box A/B of the K-assembly: tools/ablib/kbuild_base vs tools/kbuild_bench (KB_ONLY per
# kernel), alternating.  Usage: tools/kb_ab.sh [reps]
cd $(dirname "$0")/..
mkdir -p gpurun_out
out=gpurun_out/kb_ab.txt; : > $out
for r in $(seq ${1:-3}); do
  for v in base new; do
    b=./tools/kbuild_bench; [ $v = base ] && b=./tools/ablib/kbuild_base
    for k in SE SE+SE+WN; do
      KB_ONLY=$k timeout -k 10 60 $b 2>/dev/null | grep kbuild | sed "s/^/$v /" >> $out || exit 1
    done
  done
done
cat $out
