"""The benches' launch contract (bench_launch.py): `--gpus N` measures N ranks or refuses.

CPU tests: a launcher-made rank whose WORLD_SIZE differs from --gpus exits non-zero before any
GPU work, for all three benches; the GPU-free parent starts N child ranks with their own
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*, forwards rank 0's stdout only, and propagates a
failing rank's status (and ends the ranks left waiting).  GPU test: `bench.py --gpus 2` on the
one-GPU box (two ranks sharing the device over gloo) prints ONE JSON line with n_gpus = 2.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("bench", ["bench.py", "bench_split.py", "bench_mll.py"])
def test_world_size_mismatch_refused(bench):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, bench), "--gpus", "2"], env=env,
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr and r.stdout == ""


def _script(tmp_path, body):
    p = tmp_path / "rank.py"
    p.write_text(textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {ROOT!r})
        from bench_launch import spawn_ranks
        code = spawn_ranks(int(sys.argv[1]))
        if code is not None:
            sys.exit(code)
        env = {{k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE",
                                               "MASTER_ADDR", "MASTER_PORT")}}
        {body}
    """))
    return p


def test_spawn_ranks_env_and_single_stdout_line(tmp_path):
    p = _script(tmp_path, "print(json.dumps(env), flush=True)")
    r = subprocess.run([sys.executable, str(p), "3"], capture_output=True, text=True,
                       timeout=120, env={k: v for k, v in os.environ.items()
                                         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1  # rank 0's line only; ranks 1 and 2 printed to stderr
    e0 = json.loads(lines[0])
    assert e0["RANK"] == "0" and e0["LOCAL_RANK"] == "0" and e0["WORLD_SIZE"] == "3"
    assert e0["MASTER_ADDR"] == "127.0.0.1" and int(e0["MASTER_PORT"]) > 0
    others = [json.loads(x) for x in r.stderr.strip().splitlines() if x.startswith("{")]
    assert sorted(o["RANK"] for o in others) == ["1", "2"]
    assert all(o["MASTER_PORT"] == e0["MASTER_PORT"] for o in others)


def test_spawn_ranks_failure_propagates_and_ends_waiters(tmp_path):
    # rank 1 fails at once; ranks 0 and 2 would wait forever (a collective that never completes)
    body = ("import time\n        if env['RANK'] == '1': sys.exit(7)\n"
            "        time.sleep(600)")
    p = _script(tmp_path, body)
    code = ("import sys; sys.path.insert(0, %r); sys.argv = [%r, '3']; "
            "from bench_launch import spawn_ranks; "
            "sys.exit(spawn_ranks(3, argv=[%r, '3'], grace_s=1.0))" % (ROOT, str(p), str(p)))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items()
                            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 7


def test_spawn_ranks_single_gpu_is_rank_itself(tmp_path):
    p = _script(tmp_path, "print(json.dumps(env), flush=True)")
    r = subprocess.run([sys.executable, str(p), "1"], capture_output=True, text=True, timeout=60,
                       env={k: v for k, v in os.environ.items()
                            if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert r.returncode == 0
    assert json.loads(r.stdout)["WORLD_SIZE"] is None


@pytest.mark.gpu
def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` with no launcher on the one-GPU box: the parent forks two ranks
    (sharing cuda:0 over gloo), and stdout is ONE JSON line with n_gpus = 2 and the world's
    value (2 replicas' jobs/s)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--dist-backend", "gloo", "--n", "4096", "--np", "1024", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline", "--no-split-full", "--no-se-ard"],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["value"] > 0 and out["results_finite"]
    assert out["config"]["parallelism"] == "replicas x2"
    assert '"split_predict"' in r.stderr
    split = [json.loads(x) for x in r.stderr.splitlines() if x.startswith('{"split_predict"')]
    assert split and split[-1]["split_predict"]["n_gpus"] == 2, split


def test_workload_label_names_the_config():
    """bench.py labels its line with the BASELINE config it ran (review r05: the C2 run was
    labelled C3): C2 = SE-ARD N = 8192 d = 8, C3 = SE+SE+WN N = 32768 d = 8, else custom."""
    import types
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    src = open(os.path.join(ROOT, "bench.py")).read()
    ns = {}
    start = src.index("def config_label(a):")
    end = src.index("def kinds_of(name):")
    exec(compile(src[start:end], "bench.py", "exec"), ns)  # (the pure function only: no torch)
    lab = ns["config_label"]
    A = lambda k, n, d: types.SimpleNamespace(kernel=k, n=n, d=d)  # noqa: E731
    assert lab(A("SE", 8192, 8)) == "C2"
    assert lab(A("SE+SE+WN", 32768, 8)) == "C3"
    assert lab(A("SE", 32768, 8)) == "custom"
    assert lab(A("SE+SE+WN", 4096, 8)) == "custom"
    assert spec is not None
