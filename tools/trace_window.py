"""Per-stream kernel totals of the last window [first kernel matching A, first later kernel
matching B] of a rocprofv3 kernel-trace CSV.  usage: trace_window.py trace.csv A B [nshow]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"]); r["e"] = int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    r["name"] = nm.split("(")[0].split("<")[0]
    r["grid"] = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
rows.sort(key=lambda r: r["s"])
a = [i for i, r in enumerate(rows) if sys.argv[2] in r["name"]]
lo = a[-1]
hi = next(i for i in range(lo + 1, len(rows)) if sys.argv[3] in rows[i]["name"])
win = rows[lo:hi + 1]
t0 = win[0]["s"]
print("window %.2f ms, %d dispatches" % ((win[-1]["e"] - t0) / 1e6, len(win)))
by = defaultdict(lambda: defaultdict(lambda: [0, 0.0]))
for r in win:
    by[r["Stream_Id"]][(r["name"], r["grid"])][0] += 1
    by[r["Stream_Id"]][(r["name"], r["grid"])][1] += (r["e"] - r["s"]) / 1e6
for sid, kinds in by.items():
    print("stream", sid, "busy %.2f ms" % sum(v[1] for v in kinds.values()))
    for (nm, gr), (c, ms) in sorted(kinds.items(), key=lambda x: -x[1][1])[:12]:
        print("   %-36s grid %6d  x%4d  %8.3f ms  (%.3f avg)" % (nm, gr, c, ms, ms / c))
n = int(sys.argv[4]) if len(sys.argv) > 4 else 0
for r in win[:n]:
    print("%9.3f %8.3f %-32s grid=%d stream=%s" % ((r["s"] - t0) / 1e6, (r["e"] - r["s"]) / 1e6, r["name"], r["grid"], r["Stream_Id"]))
