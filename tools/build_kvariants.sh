#!/bin/bash
# Build kbuild_bench binaries for K-assembly compile-time variants: tag:defines ...
set -e
cd "$(dirname "$0")/../gaussianprocessregression.jl_amd/csrc"
make -s all build/kbuild_bench.o
OBJS="build/gpr_ctx.o build/gemm.o build/potrf.o build/mll.o build/predict.o"
for spec in "$@"; do
  tag=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $defs -c assembly.hip -o build/assembly_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -o ../../tools/kbuild_bench_$tag build/kbuild_bench.o $OBJS build/assembly_$tag.o
done
