"""Summarise a rocprofv3 kernel-trace CSV: per-stream busy time and per-kernel-kind totals for
the last potrf (the window between the last two kmat_sym_kernel dispatches)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"]); r["e"] = int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    r["name"] = nm.split("(")[0].split("<")[0]
rows.sort(key=lambda r: r["s"])
ks = [i for i, r in enumerate(rows) if "kmat_sym" in r["name"]]
lo = ks[-1] + 1
win = rows[lo:]
t0, t1 = win[0]["s"], max(r["e"] for r in win)
print(f"window {len(win)} dispatches, {(t1 - t0) / 1e6:.2f} ms")
by_stream = defaultdict(list)
for r in win:
    by_stream[r["Stream_Id"]].append(r)
for sid, rs in by_stream.items():
    busy = sum(r["e"] - r["s"] for r in rs)
    gaps = sum(max(0, rs[i + 1]["s"] - rs[i]["e"]) for i in range(len(rs) - 1))
    kinds = defaultdict(lambda: [0, 0.0])
    for r in rs:
        key = r["name"] + f" grid={int(r['Grid_Size_X']) // int(r['Workgroup_Size_X'])}" if False else r["name"]
        kinds[key][0] += 1; kinds[key][1] += (r["e"] - r["s"]) / 1e6
    print(f"stream {sid}: {len(rs)} kernels, busy {busy / 1e6:.2f} ms, gaps {gaps / 1e6:.2f} ms")
    for k, (c, ms) in sorted(kinds.items(), key=lambda x: -x[1][1]):
        print(f"    {k:40s} {c:5d} {ms:9.2f} ms")
# gemm sizes on the panel stream: classify by grid size
