"""Does SciPy's OpenBLAS dpotrf factor the C3 matrix (SE+SE+WN, N = 32768) on this host?
(In the build container scipy-openblas 0.3.28 returns info = 16545 for it; MKL factors it.)
Times the reference-order C3 job stages when it does.  Usage: python tools/cpu_potrf_probe.py [N]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import scipy.linalg as sla  # noqa: E402
from threadpoolctl import threadpool_limits  # noqa: E402

from oracle import gpr_oracle as O  # noqa: E402
from oracle.cpu_kbuild import kbuild_cpu  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
threads = int(os.environ.get("OMP_NUM_THREADS") or os.cpu_count())
kinds = [O.SE, O.SE, O.WN]
x = np.random.default_rng(0).random((8, n))
hp = O.default_hp(kinds, 8)
with threadpool_limits(limits=threads):
    for lower in (False, True):
        t0 = time.perf_counter()
        K = kbuild_cpu(kinds, hp, x)
        t1 = time.perf_counter()
        c, info = sla.lapack.dpotrf(K, lower=int(lower), clean=0, overwrite_a=1)
        t2 = time.perf_counter()
        print(f"N={n} threads={threads} uplo={'L' if lower else 'U'}: kbuild {t1 - t0:.2f} s, "
              f"dpotrf {t2 - t1:.2f} s ({n ** 3 / 3 / (t2 - t1) / 1e9:.0f} GFLOP/s), info={info}",
              flush=True)
        del K, c
