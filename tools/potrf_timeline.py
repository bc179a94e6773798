"""Timeline of the last factorisation in a rocprofv3 kernel-trace CSV (tools/gemm_bench N 0 2,
or any run whose last K-assembly is followed by a POTRF).

Per stream: busy time, idle gaps, per-kernel totals; then, for the stream carrying the
largest GEMM launches (the trailing-update stream), every launch with the idle gap before
it, so the chain-bound stretches (the trailing stream waiting for the lookahead panel)
are visible.   usage: potrf_timeline.py trace.csv [end_kernel_substring]
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
end_pat = sys.argv[2] if len(sys.argv) > 2 else None
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    r["name"] = nm.split("(")[0].split("<")[0]
    r["grid"] = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])) * \
        int(r.get("Grid_Size_Y", 1) or 1) // max(1, int(r.get("Workgroup_Size_Y", 1) or 1))
rows.sort(key=lambda r: r["s"])
ks = [i for i, r in enumerate(rows) if "kmat_sym" in r["name"]]
lo = ks[-1] + 1
hi = len(rows)
if end_pat:
    hi = next((i for i in range(lo, len(rows)) if end_pat in rows[i]["name"]), len(rows))
win = rows[lo:hi]
t0, t1 = win[0]["s"], max(r["e"] for r in win)
print(f"window: {len(win)} dispatches, {(t1 - t0) / 1e6:.3f} ms")
by = defaultdict(list)
for r in win:
    by[r["Stream_Id"]].append(r)
main = max(by, key=lambda s: max(r["e"] - r["s"] for r in by[s]))
for sid, rs in by.items():
    busy = sum(r["e"] - r["s"] for r in rs)
    gaps = sum(max(0, rs[i + 1]["s"] - rs[i]["e"]) for i in range(len(rs) - 1))
    print(f"stream {sid}{' (trailing)' if sid == main else ''}: {len(rs)} launches, "
          f"busy {busy / 1e6:.3f} ms, gaps {gaps / 1e6:.3f} ms")
    kinds = defaultdict(lambda: [0, 0.0])
    for r in rs:
        kinds[r["name"]][0] += 1
        kinds[r["name"]][1] += (r["e"] - r["s"]) / 1e6
    for k, (c, ms) in sorted(kinds.items(), key=lambda x: -x[1][1]):
        print(f"    {k:34s} {c:5d} {ms:9.3f} ms  ({ms / c * 1e3:8.1f} us avg)")
print("\ntrailing-stream launches (t from window start, ms):")
prev = t0
idle = 0
for r in by[main]:
    gap = (r["s"] - prev) / 1e6
    idle += max(0.0, gap)
    print(f"  t={(r['s'] - t0) / 1e6:8.3f}  gap {gap:7.3f}  dur {(r['e'] - r['s']) / 1e6:7.3f}  "
          f"{r['name']} grid={r['grid']}")
    prev = r["e"]
tail = (t1 - prev) / 1e6
print(f"trailing stream idle inside the window: {idle:.3f} ms + {tail:.3f} ms after its last launch")
