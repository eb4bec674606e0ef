"""bench.py's launcher path on the CPU: spawn_ranks starts N fresh gloo ranks (127.0.0.1
rendezvous, RANK / LOCAL_RANK / WORLD_SIZE set), the tile shards are gathered to rank 0 only, and
rank 0's unsharded frame equals the unsharded render; a failing rank fails the job."""
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from octree_pathtracing_amd.launch import spawn_ranks

ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("world,W,H", [(2, 40, 24), (3, 29, 21)])
def test_spawn_ranks_gathers_to_rank0(tmp_path, world, W, H):
    out = tmp_path / "frame.npy"
    rc = spawn_ranks(world, [str(ROOT / "tests" / "_launch_worker.py"), str(out), str(W), str(H)], timeout=240)
    assert rc == 0
    got, frame = np.load(out)
    assert np.array_equal(got, frame)


def test_spawn_ranks_propagates_failure():
    rc = spawn_ranks(2, ["-c", "import os, sys; sys.exit(3 if os.environ['RANK'] == '1' else 0)"], timeout=60)
    assert rc == 3


def test_bench_refuses_world_mismatch():
    """Under torchrun-style env the job's WORLD_SIZE must equal --gpus."""
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "PATH": "/usr/bin:/bin"}
    p = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "3", "--no-cpu-baseline"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "WORLD_SIZE=2" in p.stderr
