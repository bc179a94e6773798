#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only) on the K-assembly microbench:
# VALU/LDS/wait breakdown of kmat_sym2_kernel.  Usage: tools/pmc_kbuild.sh <bench-suffix> [config]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=$ROOT/tools/kbuild_bench${1:+_$1}
OUT=$ROOT/gpurun_out/pmc_kbuild${1:+_$1}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export KB_ONLY=${2:-SE+SE+WN}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o p -- $B > $OUT/p$i.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "kmat" not in k:
            continue
        agg[k[:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {sum(v)/len(v):.4g}  (n={len(v)})")
PY
