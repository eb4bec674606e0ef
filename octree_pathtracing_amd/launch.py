"""One process per GPU without torchrun: `bench.py --gpus N` started bare spawns N
fresh ranks of the same command line, each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set, and waits for them.  The parent never touches the GPU (it imports neither torch nor
liboctpt), so no process that initialised HIP is ever replaced or forked."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(nprocs: int, argv: list[str], timeout: float | None = None, env: dict | None = None) -> int:
    """Run `python argv...` as ranks 0..nprocs-1 of one job on 127.0.0.1; return the first non-zero
    exit code (the other ranks are then terminated) or 0.  stdout / stderr are inherited."""
    port = free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, *argv], env=e))
    t0 = time.monotonic()
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code  # killed by a signal
            if rc != 0:
                break
            if timeout is not None and time.monotonic() - t0 > timeout:
                rc = 124
                break
            time.sleep(0.05)
    finally:
        for p in procs:  # only our own children, by handle
            p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
    return rc
