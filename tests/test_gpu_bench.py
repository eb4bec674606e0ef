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


def _bench(tmp_path, n, extra=(), spp=("--spp", "2"), cpu=("--no-cpu-baseline",)):
    out = tmp_path / f"frame{n}.npy"
    cmd = [sys.executable, str(ROOT / "bench.py"), "--gpus", str(n), "--config", "C2", *spp, "--steps", "1",
           "--warmup", "0", *cpu, "--dump-frame", str(out), *extra]
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
    # a run at another spp than the config's quotes no committed profile (test_two_rank_line_complete quotes one)
    assert rf["traffic"] is None and rf["measured"] is None and "own frame" in rf["traffic_source"]
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


def test_two_rank_line_complete(tmp_path):
    """The N-rank line carries everything the one-GPU line does: traffic and the measured
    read / write GB/s from a profile of the same rank count (profiles/pmc_C2_n2.json, rank 0's shard), and the
    CPU baseline timed on rank 0 in the same run, after the timed steps."""
    one, f1 = _bench(tmp_path, 1, spp=(), cpu=("--cpu-seconds", "1"))
    two, f2 = _bench(tmp_path, 2, ("--dist-backend", "gloo", "--no-capi-multi"), spp=(), cpu=("--cpu-seconds", "1"))
    assert np.array_equal(f1, f2)
    for line, n in ((one, 1), (two, 2)):
        rf = line["roofline"]
        name = "pmc_C2.json" if n == 1 else "pmc_C2_n2.json"
        assert rf["traffic"] and rf["traffic"] > 0 and name in rf["traffic_source"], rf["traffic_source"]
        m = rf["measured"]
        assert m and m["source"] == f"profiles/{name}"
        assert m["read_gbs"] > 0 and m["write_gbs"] > 0
        assert m["read_frac"] == pytest.approx(m["read_gbs"] / rf["peak"], abs=1e-4)
        assert m["total_gbs"] == pytest.approx(m["read_gbs"] + m["write_gbs"], abs=0.2)
        cb = line["cpu_baseline"]
        assert cb and cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
        assert cb["gpu_over_cpu"] == pytest.approx(line["value"] / cb["value"], rel=1e-2)
    assert two["n_gpus"] == 2 and "capi_multi" not in two
