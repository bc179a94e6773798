"""Per-stream summary of one window of a rocprofv3 kernel-trace CSV: the window starts at the
k-th dispatch whose name contains START (default: the last but one) and ends at the next
dispatch containing END.   usage: trace_streams.py trace.csv START END [k] [nshow]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    r["name"] = nm.split("(")[0].split("<")[0]
    r["grid"] = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
rows.sort(key=lambda r: r["s"])
starts = [i for i, r in enumerate(rows) if sys.argv[2] in r["name"]]
k = int(sys.argv[4]) if len(sys.argv) > 4 else -2
lo = starts[k]
hi = next(i for i in range(lo + 1, len(rows)) if sys.argv[3] in rows[i]["name"])
win = rows[lo:hi + 1]
t0, t1 = win[0]["s"], max(r["e"] for r in win)
print(f"window {(t1 - t0) / 1e6:.3f} ms, {len(win)} dispatches")
by = defaultdict(list)
for r in win:
    by[r["Stream_Id"]].append(r)
for sid, rs in by.items():
    busy = sum(r["e"] - r["s"] for r in rs) / 1e6
    print(f"stream {sid}: {len(rs)} launches, busy {busy:.3f} ms, span "
          f"{(rs[0]['s'] - t0) / 1e6:.3f}..{(max(r['e'] for r in rs) - t0) / 1e6:.3f}")
    kinds = defaultdict(lambda: [0, 0.0])
    for r in rs:
        kinds[r["name"]][0] += 1
        kinds[r["name"]][1] += (r["e"] - r["s"]) / 1e6
    for nm, (c, ms) in sorted(kinds.items(), key=lambda x: -x[1][1])[:8]:
        print(f"    {nm:34s} {c:5d} {ms:9.3f} ms")
n = int(sys.argv[5]) if len(sys.argv) > 5 else 0
for r in win[:n]:
    print(f"{(r['s'] - t0) / 1e3:10.1f} us  dur {(r['e'] - r['s']) / 1e3:8.1f}  s{r['Stream_Id']} "
          f"{r['name'][:30]} grid={r['grid']}")
