"""One-process-per-GPU launcher shared by bench.py, bench_split.py and bench_mll.py.

`python bench.py --gpus N` must measure N ranks whether or not the caller used
`torch.distributed.run`:

* WORLD_SIZE set (a launcher made this process a rank): it must equal --gpus, or the run is
  refused (exit 2) -- a line whose `n_gpus` differs from what was asked for is never printed.
* WORLD_SIZE unset and --gpus N > 1: this process becomes the parent.  It never touches the
  GPU (no HIP call, no torch.cuda call: it only forks), starts N fresh child processes of the
  same script with RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR /
  MASTER_PORT set (subprocess.Popen, never exec), forwards rank 0's stdout (the ONE JSON line)
  to its own stdout, sends every other rank's stdout to stderr, and exits with the first
  non-zero child status (after ending the remaining ranks, which would otherwise wait in a
  collective forever).
* WORLD_SIZE unset and --gpus 1: nothing to do, this process is rank 0 of 1.

This module must stay GPU-free: it imports nothing from torch or gpr_amd.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def check_world(gpus: int, script: str) -> None:
    """Refuse a launcher-made rank whose WORLD_SIZE disagrees with --gpus."""
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None and int(ws) != gpus:
        sys.stderr.write(f"{script}: --gpus {gpus} but WORLD_SIZE={ws}: refusing to measure a "
                         "different number of ranks than requested\n")
        sys.exit(2)


def spawn_ranks(gpus: int, argv: list[str] | None = None, poll_s: float = 0.2,
                grace_s: float = 30.0) -> int | None:
    """Parent side of the contract above.  Returns None when this process is itself a rank
    (WORLD_SIZE set, or --gpus 1); otherwise runs the N ranks to completion and returns the
    exit status the parent should exit with."""
    script = os.path.basename(sys.argv[0] if argv is None else argv[0])
    check_world(gpus, script)
    if os.environ.get("WORLD_SIZE") is not None or gpus <= 1:
        return None
    argv = list(sys.argv if argv is None else argv)
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(gpus),
                   LOCAL_WORLD_SIZE=str(gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=port)
        # rank 0 writes the JSON line on the inherited stdout; the other ranks' stdout (RCCL
        # banners and the like) goes to stderr so stdout carries exactly one line
        out = None if r == 0 else sys.stderr.fileno()
        procs.append(subprocess.Popen([sys.executable] + argv, env=env, stdout=out,
                                      start_new_session=True))
    status = 0
    failed_at = None
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad and status == 0:
                status = bad[0] if bad[0] > 0 else 128 - bad[0]
                failed_at = time.monotonic()
            if all(c is not None for c in codes):
                break
            if failed_at is not None and time.monotonic() - failed_at > grace_s:
                # a rank failed: the survivors are waiting in a collective that never completes
                for p in procs:
                    if p.poll() is None:
                        os.killpg(p.pid, signal.SIGTERM)
                time.sleep(5.0)
                for p in procs:
                    if p.poll() is None:
                        os.killpg(p.pid, signal.SIGKILL)
                for p in procs:
                    p.wait()
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGTERM)
        for p in procs:
            p.wait()
        return 130
    return status
