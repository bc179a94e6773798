#!/bin/bash
# Run kbuild_bench variants (sym lines only).
set -e
cd "$(dirname "$0")/.."
for b in "$@"; do
  timeout -k 10 60 tools/kbuild_bench_$b 2>&1 | grep "kbuild.*sym\|kbuild.*cross" | sed "s/^/$b: /"
done
