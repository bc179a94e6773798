"""Round 6: accumulation pieces per task in the tile-DAG list-scheduling model (tools/dag_sim.py)
and the sensitivity of the job to a per-piece pipeline prologue (fill + drain).  Not a test."""
import heapq, sys
import numpy as np
sys.path.insert(0, "tools")
from dag_sim import task_list

def sim_pieces(nt, ntr, tasks, W=256, c_step=15.8, c_load=1.5, c_fac=58.0, c_tri=10.0, c_pub=2.6, prologue=0.0):
    finA = np.full((nt, nt), np.inf); finR = np.full((nt, max(ntr,1)), np.inf)
    free = [0.0]*W; heapq.heapify(free); end = 0.0
    pieces = []; small = 0; total_blocks = 0
    for kind, i, j in tasks:
        t0 = heapq.heappop(free); t = t0 + c_load
        if i > 0:
            avail = np.maximum(finA[0:i, i], finA[0:i, j] if kind == "A" else finR[0:i, j]) + c_pub
            done = 0; npc = 0
            while done < i:
                # wait until row done is available
                t = max(t, avail[done])
                r = done
                while r < i and avail[r] <= t: r += 1
                npc += 1
                nb = r - done
                if nb <= 2: small += nb
                total_blocks += nb
                t += prologue + nb * c_step
                done = r
            pieces.append(npc)
        if kind == "A" and i == j:
            t += c_fac; finA[i, i] = t
        else:
            t = max(t, finA[i, i] + c_pub) + c_tri
            if kind == "A": finA[i, j] = t
            else: finR[i, j] = t
        end = max(end, t); heapq.heappush(free, t)
    return end, np.mean(pieces), small / total_blocks

for nt, ntr, nm in ((64, 65, "C2 job"), (64, 0, "POTRF 8192"), (256, 65, "C3 job")):
    for pro in (0.0, 1.5, 3.0):
        e, mp, fs = sim_pieces(nt, ntr, task_list(nt, ntr), prologue=pro)
        print(f"{nm}: prologue {pro} us -> {e/1e3:.3f} ms, mean pieces/task {mp:.2f}, blocks in pieces<=2: {fs:.3f}")
