"""Discrete-event model of the persistent tile-DAG launch (csrc/dag.hip) to study task orders
on the CPU.  Not a test and not the product path.

Model: W workgroups take tasks in ticket order (greedy list scheduling: the next ticket goes
to the first workgroup that frees up).  A task of tile (i, j) (or right-hand-side tile (i, c))
loads its tile (c_load), accumulates row blocks k < i in order, block k not before both
inputs (tile (k, i) of A and tile (k, j) of A or B) are final (c_step per block), then
  diagonal:      factors the tile and writes W_i (c_fac)                   -> final
  off-diagonal:  waits for W_i (the diagonal task of row i), U_ij = W_i^T B (c_tri) -> final
Final tiles become visible to waiters c_pub later.  Times in microseconds.

    python tools/dag_sim.py                 (calibration against the measured launches)
"""
import argparse
import heapq

import numpy as np


def task_list(nt, ntr, rlag=0, fearly=False, lower=False, zlag=2, order="rows"):
    """The host-built ticket order of launch_potrf_dag (dag.hip), or an alternative."""
    tasks = []
    lag = min(zlag if lower else rlag, nt)

    def rhs_row(i):
        for c in range(min(ntr, i + 1) if lower else ntr):
            tasks.append(("R", i, c))

    if order == "rows":
        for i in range(nt):
            if not fearly or i == 0:
                tasks.append(("A", i, i))
            for j in range(i + 1, nt):
                tasks.append(("A", i, j))
                if fearly and j == i + 1:
                    tasks.append(("A", j, j))
            if i - lag >= 0:
                rhs_row(i - lag)
        for i in range(max(nt - lag, 0), nt):
            rhs_row(i)
    elif order.startswith("cols"):
        # right-looking-friendly: tile (i, j) in column-major order of j, then RHS by rows
        for j in range(nt):
            for i in range(j + 1):
                tasks.append(("A", i, j))
            if j - lag >= 0:
                rhs_row(j - lag)
        for i in range(max(nt - lag, 0), nt):
            rhs_row(i)
    return tasks


def simulate(nt, ntr, tasks, W=256, c_step=14.8, c_load=1.5, c_fac=48.0, c_tri=7.4, c_pub=1.5,
             lower=False, rhs_step=None, kstep=None):
    rhs_step = c_step if rhs_step is None else rhs_step
    finA = np.full((nt, nt), np.inf)
    finR = np.full((nt, max(ntr, 1)), np.inf)
    if lower:  # identity's zero tiles above the diagonal: final from the start
        for c in range(ntr):
            finR[:c, c] = 0.0
    free = [0.0] * W
    heapq.heapify(free)
    busy = 0.0
    end = 0.0
    for kind, i, j in tasks:
        t0 = heapq.heappop(free)
        t = t0 + c_load
        k0 = j if (kind == "R" and lower) else 0
        step = c_step if kind == "A" else rhs_step
        if i > k0:
            a = np.maximum(finA[k0:i, i], finA[k0:i, j] if kind == "A" else finR[k0:i, j]) + c_pub
            K = i - k0
            t = max(t + K * step, float(np.max(a + step * np.arange(K, 0, -1))))
        if kind == "A" and i == j:
            t += c_fac
            finA[i, i] = t
        else:
            t = max(t, finA[i, i] + c_pub) + c_tri
            if kind == "A":
                finA[i, j] = t
            else:
                finR[i, j] = t
        busy += t - t0
        end = max(end, t)
        heapq.heappush(free, t)
    return end, busy / (W * end)


def flops(nt, ntr, lower=False):
    n = nt * 128.0
    f = n ** 3 / 3
    f += (n ** 3 / 3 if lower else n * n * ntr * 128.0)
    return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--c-step", type=float, default=14.8)
    ap.add_argument("--c-fac", type=float, default=48.0)
    ap.add_argument("--c-tri", type=float, default=7.4)
    ap.add_argument("--c-pub", type=float, default=1.5)
    args = ap.parse_args()
    kw = dict(c_step=args.c_step, c_fac=args.c_fac, c_tri=args.c_tri, c_pub=args.c_pub)
    cases = [("POTRF N=8192", 64, 0), ("C2 job N=8192 np=8192", 64, 64),
             ("C3 job N=32768 np=8192", 256, 64), ("POTRF N=32768", 256, 0)]
    for name, nt, ntr in cases:
        for rlag in (0, 1, 2, 4):
            for fearly in (False, True):
                if ntr == 0 and rlag:
                    continue
                tl = task_list(nt, ntr, rlag=rlag, fearly=fearly)
                e, u = simulate(nt, ntr, tl, **kw)
                print(f"{name:26s} rlag={rlag} fearly={int(fearly)}: {e / 1e3:8.3f} ms  "
                      f"busy {u:.3f}  {flops(nt, ntr) / e / 1e6:6.1f} TF/s")


if __name__ == "__main__":
    main()
