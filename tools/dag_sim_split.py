"""Round 6: the tile-DAG list-scheduling model (tools/dag_sim.py) with the C2 drain split:
right-hand-side tasks of the last rows split into two ADJACENT tickets (a partial sum over row
blocks [0, h) parked in scratch, and the main task over [h, i) that adds it), so no work is
inserted ahead of the chain's tickets.  Not a test."""
import heapq, sys
import numpy as np
sys.path.insert(0, "tools")
from dag_sim import task_list, flops

def simulate(nt, ntr, tasks, W=256, c_step=14.8, c_load=1.5, c_fac=48.0, c_tri=7.4, c_pub=1.5):
    finA = np.full((nt, nt), np.inf); finR = np.full((nt, ntr), np.inf)
    finP = {}
    free = [0.0] * W; heapq.heapify(free); busy = 0.0; end = 0.0
    for task in tasks:
        kind, i, j = task[:3]
        t0 = heapq.heappop(free); t = t0 + c_load
        if kind == "P":
            h = task[3]; k0, k1 = 0, h
        elif kind == "S":
            h = task[3]; k0, k1 = h, i
        else:
            k0, k1 = 0, i
        if k1 > k0:
            src = finA[k0:k1, j] if kind == "A" else finR[k0:k1, j]
            a = np.maximum(finA[k0:k1, i], src) + c_pub
            K = k1 - k0
            t = max(t + K * c_step, float(np.max(a + c_step * np.arange(K, 0, -1))))
        if kind == "P":
            finP[(i, j)] = t
        elif kind == "A" and i == j:
            t += c_fac; finA[i, i] = t
        else:
            if kind == "S":
                t = max(t, finP[(i, j)] + c_pub) + c_load
            t = max(t, finA[i, i] + c_pub) + c_tri
            if kind == "A": finA[i, j] = t
            else: finR[i, j] = t
        busy += t - t0; end = max(end, t); heapq.heappush(free, t)
    return end, busy / (W * end)

def split_list(nt, ntr, i0, frac=0.5, adjacent=True, maxsplit=None):
    base = task_list(nt, ntr)
    out = []
    for tk in base:
        kind, i, j = tk
        if kind == "R" and i >= i0 and i >= 2:
            h = max(1, int(i * frac))
            out.append(("P", i, j, h)); out.append(("S", i, j, h))
        else:
            out.append(tk)
    return out

nt, ntr = 64, 65
e, u = simulate(nt, ntr, task_list(nt, ntr))
print(f"baseline C2: {e/1e3:.3f} ms busy {u:.3f}  {flops(nt,ntr)/e/1e6:.1f} TF/s")
for i0 in (40, 48, 52, 56, 60, 62):
    for frac in (0.3, 0.5, 0.7):
        e, u = simulate(nt, ntr, split_list(nt, ntr, i0, frac))
        print(f"split rows>={i0} frac {frac}: {e/1e3:.3f} ms busy {u:.3f}")
# C3
nt, ntr = 256, 65
e, u = simulate(nt, ntr, task_list(nt, ntr)); print(f"baseline C3: {e/1e3:.3f} ms busy {u:.3f}")
for i0 in (224, 240, 248):
    e, u = simulate(nt, ntr, split_list(nt, ntr, i0, 0.5)); print(f"C3 split rows>={i0}: {e/1e3:.3f} ms busy {u:.3f}")
print("calibrated (15.8/58/10/2.6)")
kw = dict(c_step=15.8, c_fac=58.0, c_tri=10.0, c_pub=2.6)
for nt, ntr, nm in ((64, 0, "POTRF 8192"), (64, 65, "C2 job")):
    e, u = simulate(nt, max(ntr,1), task_list(nt, ntr), **kw)
    print(f"{nm}: {e/1e3:.3f} ms busy {u:.3f}")
for i0 in (56, 60, 62):
    e, u = simulate(64, 65, split_list(64, 65, i0, 0.5), **kw); print(f"C2 split rows>={i0}: {e/1e3:.3f} ms busy {u:.3f}")
