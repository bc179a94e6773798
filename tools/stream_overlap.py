"""From a rocprofv3 kernel-trace CSV of tools/mgpu_stream_probe.py (streamed mode): for the last
potrf_dag_kernel launch, how much of the stream-out work (rows_gate/rows_pack kernels and the
RCCL broadcast kernels) ran inside the launch's [start, end] window.

  python tools/stream_overlap.py <kernel_trace.csv>
"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    dags = [x for x in k if "potrf_dag_kernel" in x[0]]
    s0, e0 = dags[-1][1], dags[-1][2]
    prev_end = max([x[2] for x in dags[:-1]], default=0)
    out = [x for x in k if x[1] >= prev_end and ("rows_" in x[0] or "ncclDevKernel" in x[0]
                                                or "nccl" in x[0].lower())]
    print(f"last DAG launch: {(e0 - s0) / 1e6:.2f} ms")
    inside = sum(max(0, min(e, e0) - max(s, s0)) for _, s, e in out)
    total = sum(e - s for _, s, e in out)
    last_end = max((e for _, s, e in out), default=e0)
    by = {}
    for n, s, e in out:
        m = re.search(r"(rows_\w+(<\w+>)?|nccl\w+)", n)
        key = m.group(1) if m else n[:60]
        c = by.setdefault(key, [0, 0, 0])
        c[0] += 1
        c[1] += e - s
        c[2] += max(0, min(e, e0) - max(s, s0))
    for key, (cnt, t, ins) in sorted(by.items()):
        print(f"  {key:60s} x{cnt:3d}  {t / 1e6:8.3f} ms busy, {ins / 1e6:8.3f} ms inside the DAG window")
    print(f"stream-out kernels: {total / 1e6:.3f} ms busy, {inside / 1e6:.3f} ms inside the DAG window; "
          f"last one ends {(last_end - e0) / 1e6:.3f} ms after the DAG")


if __name__ == "__main__":
    main()
