"""One rank of the multi-process C5 parity test (test_gpu_fullsize_oracle.py
test_c5_split_predict_distributed_rccl_vs_oracle_fixture): split_predict_distributed over an
RCCL (backend "nccl") process group, one process per GPU -- the path bench.py's C5 leg and the
SCALE runs measure -- for both fit modes, checked on every rank against the committed C5 oracle
fixture (tests/golden/fullsize_C5.npz) at the tolerances of the single-device test
(src/split_predict.jl:5-53 is the reference).

    RANK=r WORLD_SIZE=n LOCAL_RANK=r MASTER_ADDR=127.0.0.1 MASTER_PORT=p python dist_c5_worker.py

Prints "OK rank r" and exits 0 when every check passes on this rank.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(HERE, "golden"), ROOT, os.path.join(ROOT, "gaussianprocessregression.jl_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import make_fullsize as MF  # noqa: E402
from oracle import gpr_oracle as O  # noqa: E402  (the checker)


def main():
    rank = int(os.environ["RANK"])
    local = int(os.environ["LOCAL_RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(local)
    dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    try:
        import gpr_amd as G
        from gpr_amd.distributed import split_predict_distributed

        cfg = MF.CONFIGS["C5"]
        fx = np.load(MF.fixture_path("C5"))  # plain arrays (allow_pickle=False)
        inp = MF.inputs(cfg)
        keys = [k for k in ("x", "y", "xp", "xe", "xq") if k in inp]
        assert str(fx["input_sha256"]) == MF.checksum([inp[k] for k in keys]), "inputs changed"
        kinds, hp = cfg["kinds"], inp["hp"]
        md = G.GPRModel(G.SquaredExp() + G.WhiteNoise(), hp, inp["x"], inp["y"],
                        ctx=G.Context(local))
        assert kinds == [O.SE, O.WN]
        cm = G.Cmap("+", inp["xe"], inp["xq"])
        prior = O.diag_prior(kinds, hp, cfg["d"])
        lo, hi = cfg["var_range"]
        nq = cfg["nq"]
        rows = fx["rows"]
        for fit in ("broadcast", "replicate"):
            mu, var = split_predict_distributed(md, cm, var_range=cfg["var_range"], fit=fit)
            np.testing.assert_allclose(mu[rows], fx["mu_rows"], rtol=1e-8, atol=1e-10)
            rel = np.linalg.norm(mu[rows] - fx["mu_rows"]) / np.linalg.norm(fx["mu_rows"])
            assert rel <= 1e-8, (fit, rel)
            np.testing.assert_allclose(var[(lo - 1) * nq:hi * nq], fx["var_head"], rtol=1e-8,
                                       atol=1e-8 * prior)
            assert np.all(var[hi * nq:] == prior), fit
        dist.barrier()
        print(f"OK rank {rank} of {world}", flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
