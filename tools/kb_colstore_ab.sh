set -o pipefail
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for cs in 1 0; do
    echo "== GPR_KBUILD_COLSTORE=$cs round $r"
    GPR_KBUILD_COLSTORE=$cs KB_ONLY=SE timeout -k 10 100 ./tools/kbuild_bench | grep kbuild || exit 1
  done
done
GPR_KBUILD_COLSTORE=1 KB_ONLY=SE timeout -k 10 100 ./tools/kbuild_bench_nostore | grep kbuild
