# XCD-aware K-build item order: timing A/B (GPR_KBUILD_XCD 0/1), FETCH_SIZE per launch, parity
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
out=gpurun_out/kb_xcd_r04l.txt; : > $out
for rep in 1 2; do for x in 0 1; do for c in SE SE+SE+WN; do
  echo "== XCD=$x $c" >> $out
  GPR_KBUILD_XCD=$x KB_ONLY=$c timeout -k 10 120 ./tools/kbuild_bench 32768 8 >> $out 2>&1 || exit 1
done; done; done
for x in 0 1; do
  GPR_KBUILD_XCD=$x KB_ONLY=SE+SE+WN timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/kb_fetch_$x -o p -- ./tools/kbuild_bench 32768 8 > gpurun_out/kb_fetch_$x.log 2>&1 || exit 1
done
python3 - <<'PY' >> $out
import csv, glob
for x in (0, 1):
    f = glob.glob(f"gpurun_out/kb_fetch_{x}/**/*counter_collection.csv", recursive=True)[0]
    agg = {}
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        agg.setdefault(k, []).append(float(r["Counter_Value"]))
    for k, v in agg.items():
        if "kmat" in k:
            print(f"XCD={x} {k}: FETCH_SIZE {sum(v)/len(v):.0f} KB avg over {len(v)} (x2 for the gfx950 16-B correction)")
PY
cat $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread -k "buffer or kernel" > gpurun_out/tests_r04l.log 2>&1
rc=$?; tail -3 gpurun_out/tests_r04l.log; exit $rc
