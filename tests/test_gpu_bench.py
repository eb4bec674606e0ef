"""bench.py's N-rank path on one GPU: `--gpus 2` spawns two ranks itself, each renders
its 8x8-tile shard through liboctpt on the GPU, the shards are gathered to rank 0 (gloo, host-staged:
two ranks share this box's one GPU, which RCCL does not allow) and unsharded by the kernel.  The
gathered frame must equal the one-rank frame bit for bit and the JSON line must report n_gpus 2."""
import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _bench(tmp_path, n, extra=()):
    out = tmp_path / f"frame{n}.npy"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--config", "C2", "--spp", "2", "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--dump-frame", str(out), *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    return line, np.load(out)


def test_two_ranks_gather_equals_one(tmp_path):
    one, f1 = _bench(tmp_path, 1)
    # one warmup step: its per-tile segment counts give the balanced tile deal of the timed step
    two, f2 = _bench(tmp_path, 2, ("--dist-backend", "gloo", "--warmup", "1", "--balance"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["parallelism"] == "tiles2-gloo" and two["config"]["tile_deal"].startswith("balanced")
    assert f1.shape == f2.shape == (1280 * 720, 4)
    assert np.array_equal(f1, f2)
    # every rank's segments are counted once
    assert one["config"]["segments_per_step"] == two["config"]["segments_per_step"]
    # the N-rank roofline: per-rank figures, the aggregate is their sum over the slowest
    # rank's extend time, achieved their mean, and no one-GPU PMC traffic on a two-rank line
    rf = two["roofline"]
    ranks = rf["ranks"]
    assert [x["rank"] for x in ranks] == [0, 1] and all(x["bytes"] > 0 and x["ext_ms"] > 0 for x in ranks)
    tmax = max(x["ext_ms"] for x in ranks) / 1e3
    assert rf["aggregate_gbs"] == pytest.approx(sum(x["bytes"] for x in ranks) / tmax / 1e9, rel=1e-3)
    assert rf["achieved"] == pytest.approx(sum(x["achieved"] for x in ranks) / 2, rel=1e-3)
    assert rf["aggregate_peak"] == 2 * rf["peak"] and rf["frac_min"] <= rf["frac"] <= rf["frac_max"]
    assert rf["traffic"] is None and "pmc_C2_n2.json" in rf["traffic_source"]
    assert one["roofline"]["achieved"] > 0 and "ranks" not in one["roofline"]
    # rank 0's measurement of the same frame through one multi-device context (octpt_create_multi):
    # on this box its two entries repeat device 0
    cm = two["capi_multi"]
    assert "error" not in cm, cm
    assert cm["devices"] == [0, 0] and cm["segments"] == one["config"]["segments_per_step"] and cm["value"] > 0


def test_capi_devices_bench(tmp_path):
    """bench.py --capi-devices 2: the whole frame through one two-entry context equals the one-context frame."""
    one, f1 = _bench(tmp_path, 1)
    two, f2 = _bench(tmp_path, 1, ("--capi-devices", "2"))
    assert two["config"]["parallelism"] == "capi-multi2" and two["config"]["capi_devices"] == [0, 0]
    assert np.array_equal(f1, f2)
    assert one["config"]["segments_per_step"] == two["config"]["segments_per_step"]
