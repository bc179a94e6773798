"""Summarise a round's rocprofv3 passes of bench.py into profiles/rNN_pmc_summary.json.

Inputs (written by tools/profile_round.sh): <dir>/fetch/**/*counter_collection.csv and
<dir>/write/**/*counter_collection.csv (one --pmc pass each) and <dir>/trace/**/*kernel_stats.csv.
Per kernel name: mean FETCH_SIZE and WRITE_SIZE per dispatch (rocprofv3 reports KiB),
FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests of 16-B/lane
streaming reads at 64 B), plus the kernel-trace average duration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    s = name.replace("(anonymous namespace)::", "").strip()
    if s.startswith("void "):
        s = s[5:]
    return s.split("(")[0].split("<")[0].split("::")[-1].strip()


def per_dispatch(pattern, counter):
    tot, cnt = defaultdict(float), defaultdict(set)
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = short(r["Kernel_Name"])
            tot[name] += float(r["Counter_Value"])
            cnt[name].add(r["Dispatch_Id"])
    return {k: tot[k] / max(len(cnt[k]), 1) for k in tot}, {k: len(v) for k, v in cnt.items()}


def per_dispatch_list(pattern, counter):
    """{kernel: [counter sum of each dispatch, in dispatch order]}"""
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                vals[short(r["Kernel_Name"])][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {k: [v[i] for i in sorted(v)] for k, v in vals.items()}


def trace_stats(pattern):
    out = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            name = short(r["Name"])
            out[name] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
                         "total_ms": float(r["TotalDurationNs"]) / 1e6}
    return out


def main():
    d, n, npred = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    fetch, nf = per_dispatch(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    write, nw = per_dispatch(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    stats = trace_stats(os.path.join(d, "trace", "**", "*kernel_stats.csv"))
    # per-dispatch traffic, the two passes paired by dispatch order (same command): a kernel
    # launched with different work per call (the tile-DAG: fit + posterior solve in the job,
    # factorisation alone in the stage breakdown) is characterised by its largest launch too
    fl = per_dispatch_list(os.path.join(d, "fetch", "**", "*counter_collection.csv"), "FETCH_SIZE")
    wl = per_dispatch_list(os.path.join(d, "write", "**", "*counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        fb = 2.0 * fetch.get(k, 0.0) * 1024.0
        wb = write.get(k, 0.0) * 1024.0
        kernels[k] = {"dispatches_fetch_pass": nf.get(k, 0), "dispatches_write_pass": nw.get(k, 0),
                      "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                      "traffic_bytes_per_launch": fb + wb, "trace": stats.get(k)}
        f1, w1 = fl.get(k, []), wl.get(k, [])
        if f1 and len(f1) == len(w1):
            per = [2.0 * a * 1024.0 + b * 1024.0 for a, b in zip(f1, w1)]
            kernels[k]["traffic_bytes_each_launch"] = per
            kernels[k]["traffic_bytes_max_launch"] = max(per)
    # MFMA pass (optional): raw counters of each kernel's largest launch (by GRBM_GUI_ACTIVE),
    # plus BUSY / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs): MFMA-busy cycles per CU-cycle
    mpat = os.path.join(d, "mfma", "**", "*counter_collection.csv")
    if glob.glob(mpat, recursive=True):
        names = set()
        for f in glob.glob(mpat, recursive=True):
            names |= {r["Counter_Name"] for r in csv.DictReader(open(f))}
        lists = {c: per_dispatch_list(mpat, c) for c in sorted(names)}
        durs = defaultdict(dict)  # kernel -> {dispatch: ns}
        for f in glob.glob(mpat, recursive=True):
            for r in csv.DictReader(open(f)):
                durs[short(r["Kernel_Name"])][int(r["Dispatch_Id"])] = \
                    int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for k in set(lists.get("GRBM_GUI_ACTIVE", {})):
            g = lists["GRBM_GUI_ACTIVE"][k]
            i = max(range(len(g)), key=lambda j: g[j])
            m = {c: lists[c][k][i] for c in lists if k in lists[c] and len(lists[c][k]) == len(g)}
            busy = m.get("SQ_VALU_MFMA_BUSY_CYCLES")
            if busy is not None and g[i] > 0:
                m["mfma_busy_per_cu_cycle"] = busy / (g[i] / 8.0 * 256.0)
            dl = [durs[k][x] for x in sorted(durs[k])]
            if len(dl) == len(g) and dl[i] > 0:
                m["duration_ns"] = dl[i]
                m["clock_GHz"] = g[i] / 8.0 / dl[i]  # GRBM_GUI_ACTIVE sums the 8 XCDs
                if "SQ_INSTS_VALU_MFMA_F64" in m:  # every F64 MFMA here is 16x16x4: 2048 flop
                    m["mfma_f64_TFLOPs"] = m["SQ_INSTS_VALU_MFMA_F64"] * 2048.0 / dl[i] / 1e3
            m["dispatches"] = len(g)
            kernels.setdefault(k, {})["mfma_largest_launch"] = m
    out = {"config": {"N": n, "np": npred},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                     "`bench.py --steps 1 --warmup 0 --no-cpu-baseline`; FETCH_SIZE x2 (gfx950 "
                     "16-B/lane correction), KiB -> bytes; WRITE_SIZE of 8-B/lane stores is "
                     "uncalibrated (MI355X_MICROARCH.md, HBM section)",
           "kernels": kernels}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
