#!/bin/bash
# A/B of the tile-DAG solve modes on one box: C3 stage breakdown (posterior = solve from a
# finished factor), C4 (Z inside the DAG launch or after it), C5 var rows.
cd $(dirname "$0")/..
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "potri or fit_kinv or predict_vs" --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -1 gpurun_out/ab_tests.log; [ $rc -ne 0 ] && exit $rc
p() { python3 -c "import json,sys;d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1];print(sys.argv[2], round(d['ms_per_step'],2), {k:round(v,2) for k,v in (d.get('stage_ms_unfused') or {}).items()})" $1 "$2"; }
for s in 0 1; do
  GPR_DAG_SOLVE=$s timeout -k 10 200 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/ab_c3_$s.json 2>/dev/null || exit 1; p gpurun_out/ab_c3_$s.json "C3 solve=$s"
done
for f in 0 1; do for s in 0 1; do
  GPR_FUSE_KINV=$f GPR_DAG_SOLVE=$s timeout -k 10 200 python bench_mll.py > gpurun_out/ab_c4_$f$s.json 2>/dev/null || exit 1; p gpurun_out/ab_c4_$f$s.json "C4 fuse=$f solve=$s"
done; done
for s in 0 1; do
  GPR_DAG_SOLVE=$s timeout -k 10 300 python bench_split.py > gpurun_out/ab_c5_$s.json 2>/dev/null || exit 1; p gpurun_out/ab_c5_$s.json "C5 solve=$s"
done
