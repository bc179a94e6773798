set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
export KB_ONLY=SE+SE+WN
mkdir -p $R/gpurun_out/pmcg
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CU_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" "SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  for v in "" "GPR_KBUILD_EXACT=1"; do
    env $v timeout -s KILL 60 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcg/p$i${v:+x} -o p -- $R/tools/kbuild_bench > /dev/null 2>&1
  done
done
python3 - <<'PY'
import csv, glob, collections, os
R=os.environ["GRAFT_REPO_ROOT"]
for tag in ["", "x"]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(R + "/gpurun_out/pmcg/p[0-9]" + tag + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "sym" in k:
                agg[k[:45]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        print(tag or "gram", k, {c: "%.4g" % (sum(v) / len(v)) for c, v in sorted(d.items())})
PY
