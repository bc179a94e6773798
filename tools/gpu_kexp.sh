#!/bin/bash
# K-assembly exp variants (GPR_KEXP_VARIANT 0/1/2) and compute-only / exp-free references.
set -e
cd "$(dirname "$0")/.."
for b in kbuild_bench kbuild_bench_e1 kbuild_bench_e2 kbuild_bench_nostore kbuild_bench_noexp; do
  timeout -k 10 60 tools/$b 2>&1 | grep "kbuild" | sed "s/^/$b: /"
done
