"""Summarise the K-assembly PMC passes of tools/gpu_r05e.sh (rocprofv3 rocpd databases under
gpurun_out/kpmc/p1..p4, kernel trace under tr) into profiles/r05_kbuild_pmc.txt.

Per (kernel, call) group -- kbuild_bench launches kmat_symu_kernel 4 times for the full
symmetric K, then 6 times for the fit's upper-only K; the ordinal of a dispatch among its
kernel's dispatches tells them apart -- mean per dispatch of every counter collected (rows of one dispatch
summed), the kernel-trace mean duration, and derived figures:
  clock      = GRBM_GUI_ACTIVE / 8 / duration (MI355X_MICROARCH.md, DVFS give-back)
  VALU/elt   = SQ_INSTS_VALU * 64 / elements written   (lane-instructions per K entry)
  MFMA F64   = SQ_INSTS_VALU_MFMA_F64 per dispatch
  VALU busy  = SQ_ACTIVE_INST_VALU * 4 / (SQ_BUSY_CU_CYCLES * 4 * 4 SIMDs)  (quad-cycles)
  write GB   = WRITE_SIZE (KiB) * 1024;  fetch GB = FETCH_SIZE (KiB) * 1024 * 2 (gfx950
               streaming-read correction of the guide).
Not a test."""
import glob
import sqlite3
import sys
from collections import defaultdict

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kpmc"


def short(name):
    s = name.replace("(anonymous namespace)::", "").strip()
    if s.startswith("void "):
        s = s[5:]
    return s.split("(")[0].split("<")[0].split("::")[-1].strip()


def label(name, ordinal):
    if name == "kmat_symu_kernel":
        return "symmetric full" if ordinal < 4 else "upper-only (fit)"
    if name == "kmat_crossg_kernel":
        return "cross"
    return ""


def load(pass_dir):
    f = glob.glob(f"{D}/{pass_dir}/**/*.db", recursive=True)
    if not f:
        return {}
    c = sqlite3.connect(f[0])
    per = defaultdict(lambda: defaultdict(float))  # (dispatch) -> counter -> value
    meta = {}
    for disp, kname, cname, val, dur in c.execute(
            "select dispatch_id, kernel_name, counter_name, value, duration "
            "from counters_collection order by dispatch_id"):
        per[disp][cname] += val
        meta[disp] = (short(kname), dur)
    seen = defaultdict(int)
    for disp in sorted(meta):
        name, dur = meta[disp]
        meta[disp] = (name, label(name, seen[name]), dur)
        seen[name] += 1
    return per, meta


def trace(pass_dir):
    f = glob.glob(f"{D}/{pass_dir}/**/*.db", recursive=True)
    c = sqlite3.connect(f[0])
    g = defaultdict(list)
    seen = defaultdict(int)
    for name, dur in c.execute("select name, duration from kernels order by dispatch_id"):
        n = short(name)
        g[(n, label(n, seen[n]))].append(dur)
        seen[n] += 1
    return g


def main():
    groups = defaultdict(lambda: defaultdict(list))
    for p in ("p1", "p2", "p3", "p4"):
        r = load(p)
        if not r:
            continue
        per, meta = r
        for disp, cs in per.items():
            k = meta[disp][:2]
            for cname, v in cs.items():
                groups[k][cname].append(v)
            if "GRBM_GUI_ACTIVE" in cs:
                groups[k]["_clock_GHz"].append(cs["GRBM_GUI_ACTIVE"] / 8 / meta[disp][2])
    tr = trace("tr")
    out = []
    for k in sorted(groups, key=lambda k: -max(tr.get(k, [0]))):
        name, what = k
        if name.startswith("__amd") or not tr.get(k) or not what:
            continue
        durs = tr[k]
        dur_ns = sorted(durs)[len(durs) // 2]
        cs = {c: sum(v) / len(v) for c, v in groups[k].items()}
        out.append(f"{name} [{what}] dispatches={len(durs)} median duration {dur_ns / 1e6:.3f} ms (kernel trace)")
        for c in sorted(x for x in cs if not x.startswith("_")):
            out.append(f"    {c:28s} {cs[c]:.4g}")
        if "_clock_GHz" in cs:
            out.append(f"    -> clock {cs['_clock_GHz']:.2f} GHz (GRBM_GUI_ACTIVE / 8 / the profiled dispatch's duration)")
        if "WRITE_SIZE" in cs:
            out.append(f"    -> HBM write {cs['WRITE_SIZE'] * 1024 / 1e9:.3f} GB, "
                       f"{cs['WRITE_SIZE'] * 1024 / dur_ns:.0f} GB/s")
        if "FETCH_SIZE" in cs:
            out.append(f"    -> HBM fetch {2 * cs['FETCH_SIZE'] * 1024 / 1e9:.3f} GB (x2 gfx950 correction)")
        if "SQ_ACTIVE_INST_VALU" in cs and "SQ_BUSY_CU_CYCLES" in cs:
            out.append(f"    -> SQ_ACTIVE_INST_VALU / SQ_BUSY_CU_CYCLES = "
                       f"{cs['SQ_ACTIVE_INST_VALU'] / cs['SQ_BUSY_CU_CYCLES']:.3f} (wave quad-cycles issuing VALU per CU busy quad-cycle)")
        if "SQ_WAIT_INST_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            out.append(f"    -> SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES = {cs['SQ_WAIT_INST_ANY'] / cs['SQ_WAVE_CYCLES']:.3f}")
        if "SQ_INSTS_VALU_MFMA_F64" in cs and "SQ_INSTS_VALU" in cs:
            out.append(f"    -> MFMA share of VALU instructions {cs['SQ_INSTS_VALU_MFMA_F64'] / cs['SQ_INSTS_VALU']:.3f}")
    print("\n".join(out))


if __name__ == "__main__":
    main()
