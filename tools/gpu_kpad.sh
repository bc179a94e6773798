#!/bin/bash
# K-assembly / store-pattern timings with a padded column stride (KB_LDPAD doubles per column)
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for p in 0 16 64 256; do
  KB_LDPAD=$p timeout -k 10 120 tools/kbuild_bench > gpurun_out/kpad_$p.txt 2>&1 || exit 1
done
echo kpad done
