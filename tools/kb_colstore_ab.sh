# A/B of the single-part upper K build's store shape (GPR_KBUILD_COLSTORE) and grid (persistent
# vs one item per wave: tools/kbuild_bench_flatgrid), SE, N = 32768, d = 8; plus the pure-store
# ceilings (tools/store_probe.py) on the same box.
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for cs in 1 0; do
    echo "== GPR_KBUILD_COLSTORE=$cs round $r (persistent grid)"
    GPR_KBUILD_COLSTORE=$cs KB_ONLY=SE timeout -k 10 100 ./tools/kbuild_bench | grep upper || exit 1
    echo "== GPR_KBUILD_COLSTORE=$cs round $r (one item per wave)"
    GPR_KBUILD_COLSTORE=$cs KB_ONLY=SE timeout -k 10 100 ./tools/kbuild_bench_flatgrid | grep upper || exit 1
  done
done
timeout -k 10 100 python3 tools/store_probe.py || exit 2
