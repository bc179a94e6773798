import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gaussianprocessregression.jl_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture
def knobs():
    """Set library knobs (include/gpr_hip.h) on the default context for one test:
    ``knobs("GPR_QUAD_EIGEN", 1)``; every changed knob gets its old value back afterwards.
    (The library reads its GPR_* environment once per context, at creation.)"""
    import gpr_amd as G
    from gpr_amd import core
    ctx = core.default_context()
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = ctx.get_knob(name)
        ctx.set_knob(name, value)

    yield set_
    for name, value in saved.items():
        ctx.set_knob(name, value)


TESTING_LIB = os.path.join(PKG, "gpr_amd", "libgpr_hip_testing.so")


def run_fault_scenario(name, *args, timeout=300):
    """Run tests/fault_scenarios.py <name> in a child process on the test build of the library
    (fault injection is compiled only into libgpr_hip_testing.so)."""
    import subprocess
    assert os.path.exists(TESTING_LIB), "build it: make -C gaussianprocessregression.jl_amd/csrc"
    env = dict(os.environ, GPR_HIP_LIB=TESTING_LIB)
    for k in ("GPR_DAG_SPIN_LIMIT", "GPR_MGPU_GATE_LIMIT", "GPR_MGPU_FAIL_UNPACK",
              "GPR_TRD_FAIL_STEP", "GPR_TRD_SPIN_LIMIT", "GPR_TRD_QCHUNK",
              "GPR_TRD_DF", "GPR_TRD_DF_TAIL", "GPR_TRD_DELAY"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "fault_scenarios.py"), name,
                        *map(str, args)], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0 and "OK" in r.stdout, \
        f"scenario {name}{args} failed (rc {r.returncode}):\n{r.stdout[-3000:]}\n{r.stderr[-3000:]}"
