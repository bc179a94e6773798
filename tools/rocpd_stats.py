"""Kernel statistics from a rocprofv3 rocpd database (the --kernel-trace --stats summary,
written as CSV): Name, Calls, TotalDurationNs, AverageNs, MinNs, MaxNs, Percentage.

  python tools/rocpd_stats.py gpurun_out/eigprof > profiles/r05_eig_kernel_stats.csv

Not a test."""
import csv
import glob
import sqlite3
import sys
from collections import defaultdict


def main():
    d = sys.argv[1]
    f = glob.glob(f"{d}/**/*.db", recursive=True) or glob.glob(d)
    durs = defaultdict(list)
    for db in f:
        c = sqlite3.connect(db)
        for name, dur in c.execute("select name, duration from kernels"):
            durs[name].append(dur)
    tot = sum(sum(v) for v in durs.values()) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for name, v in sorted(durs.items(), key=lambda kv: -sum(kv[1])):
        w.writerow([name, len(v), sum(v), f"{sum(v) / len(v):.1f}", min(v), max(v),
                    f"{100.0 * sum(v) / tot:.2f}"])


if __name__ == "__main__":
    main()
