# A/B: the SE+SE+WN upper build (kmat_symu_kernel<2, 2>) on the persistent grid vs one item per
# wave (tools/kbuild_bench_flatgrid), N = 32768, d = 8, two rounds on one box.
set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  echo "== round $r persistent"; KB_ONLY=SE+SE+WN timeout -k 10 100 ./tools/kbuild_bench | grep upper || exit 1
  echo "== round $r one item per wave"; KB_ONLY=SE+SE+WN timeout -k 10 100 ./tools/kbuild_bench_flatgrid | grep upper || exit 1
done
