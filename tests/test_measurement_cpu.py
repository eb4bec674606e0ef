"""The measurement plumbing on the CPU: bench.py's algorithmic byte
counts and traffic loading, and scripts/pmc_traffic.py's per-launch traffic and L2 hit rate from
rocprofv3 counter CSVs (synthetic files in rocprofv3's column layout)."""
import csv
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

COLS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size", "Kernel_Id",
        "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count",
        "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
EXT = "void octpt::(anonymous namespace)::wf_extend_kernel<0>(octpt::DevScene, octpt::WaveBuffers, unsigned int, " \
      "unsigned int, unsigned long long*)"
SHADE = "void octpt::(anonymous namespace)::wf_shade_kernel<false, true>(octpt::DevScene, ...)"


def _csv(d: Path, rows):
    d.mkdir(parents=True)
    with open(d / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLS)
        w.writeheader()
        for i, (kernel, counter, value) in enumerate(rows):
            r = dict.fromkeys(COLS, 0)
            r.update(Correlation_Id=i + 1, Dispatch_Id=i + 1, Agent_Id="Agent 2", Kernel_Name=kernel,
                     Counter_Name=counter, Counter_Value=value)
            w.writerow(r)


def test_pmc_traffic_per_launch_and_l2(tmp_path):
    # two extend launches and one shade launch; the runtime's own copy kernel is ignored
    _csv(tmp_path / "fetch", [("__amd_rocclr_copyBuffer", "FETCH_SIZE", 9.0), (EXT, "FETCH_SIZE", 1000.0),
                              (SHADE, "FETCH_SIZE", 50.0), (EXT, "FETCH_SIZE", 3000.0)])
    _csv(tmp_path / "write", [(EXT, "WRITE_SIZE", 10.0), (SHADE, "WRITE_SIZE", 20.0), (EXT, "WRITE_SIZE", 30.0)])
    _csv(tmp_path / "tcc", [(EXT, "TCC_HIT_sum", 90.0), (EXT, "TCC_MISS_sum", 10.0), (EXT, "TCC_HIT_sum", 60.0),
                            (EXT, "TCC_MISS_sum", 40.0), (SHADE, "TCC_HIT_sum", 1.0), (SHADE, "TCC_MISS_sum", 3.0)])
    out = tmp_path / "pmc.json"
    subprocess.run([sys.executable, str(ROOT / "scripts" / "pmc_traffic.py"), str(tmp_path / "fetch"),
                    str(tmp_path / "write"), "CX", str(out), "1.0", "test", str(tmp_path / "tcc")], check=True,
                   capture_output=True)
    d = json.loads(out.read_text())
    e = d["wf_extend_kernel"]
    assert e["launches"] == 2
    assert e["fetch_bytes_per_launch"] == 2000 * 1024 and e["write_bytes_per_launch"] == 20 * 1024
    assert e["bytes_per_launch"] == 2020 * 1024
    assert e["l2_hit_rate"] == pytest.approx(150.0 / 200.0)
    assert d["wf_shade_kernel"]["l2_hit_rate"] == pytest.approx(0.25)
    assert d["fetch_factor"] == 1.0
    # the guide's halving (factor 2) doubles the fetch bytes only
    subprocess.run([sys.executable, str(ROOT / "scripts" / "pmc_traffic.py"), str(tmp_path / "fetch"),
                    str(tmp_path / "write"), "CX", str(out)], check=True, capture_output=True)
    e2 = json.loads(out.read_text())["wf_extend_kernel"]
    assert e2["fetch_bytes_per_launch"] == 2 * e["fetch_bytes_per_launch"] and "l2_hit_rate" not in e2


def test_bench_byte_counts():
    import bench

    st = {"esvo_steps": 1000, "sphere_tests": 10, "cuboid_tests": 5, "segments": 7, "shade_events": 3,
          "texel_reads": 2, "paths": 4}
    assert bench.extend_bytes(st) == 8 * 1000 + 20 * 10 + 28 * 5
    assert bench.extend_queue_bytes(st) == 40 * 7
    assert bench.shade_bytes(st) == 152 * 7 + 68 * 3 + 4 * 2 + 16 * 4
    assert bench.shade_bytes(st, lean=True) == 120 * 7 + 68 * 3 + 4 * 2 + 16 * 4  # the 24-B path state
    # material records read from LDS are not global-memory bytes
    assert bench.shade_bytes(st, lean=True, lds_tables=True) == 120 * 7 + 20 * 3 + 4 * 2 + 16 * 4
    # the drain kernel's share (octpt_stats.drain) is not extend's
    st["drain"] = {"esvo_steps": 100, "sphere_tests": 1, "cuboid_tests": 0, "segments": 2}
    assert bench.extend_bytes(st) == 8 * 900 + 20 * 9 + 28 * 5
    assert bench.extend_queue_bytes(st) == 40 * 5


def test_bench_lean_state_rule(monkeypatch):
    """The bench's shade byte model follows the library's lean-state rule."""
    import bench
    from octree_pathtracing_amd import scene as S

    sc, _, _ = S.make_config("tiny")
    st = {"pool_slots": 100, "chunk_items": 100}
    monkeypatch.delenv("OCTPT_LEAN", raising=False)
    assert bench.lean_state(sc, st)
    assert not bench.lean_state(sc, {"pool_slots": 99, "chunk_items": 100})  # regeneration: the 40-B state
    monkeypatch.setenv("OCTPT_LEAN", "0")
    assert not bench.lean_state(sc, st)
    monkeypatch.delenv("OCTPT_LEAN")
    sc.materials[1].emittance = 5.0
    sc.emitters_enabled = True
    assert not bench.lean_state(sc, st)
    sc.emitters_enabled = False
    assert bench.lean_state(sc, st)
    S.with_sun_variant(sc, "fast")
    assert sc.strategy.sun_sampling and not bench.lean_state(sc, st)


def test_bench_loads_committed_traffic():
    import bench

    traffic, src, l2 = bench.load_traffic("C3")
    assert traffic and traffic > 0 and "pmc_C3.json" in src
    assert l2 is None or 0.0 < l2 < 1.0
    t, why, l2 = bench.load_traffic("no-such-config")
    assert t is None and l2 is None and "no PMC profile" in why
    # a line at N ranks never quotes the one-GPU profile
    t8, why8, _ = bench.load_traffic("C3", 8)
    if not (ROOT / "profiles" / "pmc_C3_n8.json").exists():
        assert t8 is None and "pmc_C3_n8.json" in why8
    else:
        assert t8 != traffic and "pmc_C3_n8.json" in why8
    h = bench.host_cpu()
    assert h["threads"] >= 1 and h["affinity"] >= 1 and h["model"]


def test_roofline_over_ranks():
    """The N-rank line's extend roofline: per-GPU mean, aggregate over the slowest rank's
    time, per-rank spread; one rank reduces to bytes / time."""
    import bench

    one = bench.roofline_over_ranks([{"bytes": 8e12, "ext_ms": 2000.0, "launches": 9}])
    assert one["achieved"] == 4000.0 and one["frac"] == 0.5 and one["aggregate_gbs"] == 4000.0
    assert one["aggregate_peak"] == 8000.0 and one["frac_min"] == one["frac_max"] == 0.5
    r = bench.roofline_over_ranks([{"bytes": 4e12, "ext_ms": 1000.0, "launches": 9},
                                   {"bytes": 3e12, "ext_ms": 1500.0, "launches": 9}])
    assert r["achieved"] == (4000.0 + 2000.0) / 2 and r["frac"] == 0.375
    assert r["aggregate_gbs"] == round(7e12 / 1.5 / 1e9, 1) and r["aggregate_peak"] == 16000.0
    assert r["frac_min"] == 0.25 and r["frac_max"] == 0.5
    assert sum(x["bytes"] for x in r["per_rank"]) == 7e12 and [x["rank"] for x in r["per_rank"]] == [0, 1]


def test_measured_rates_from_same_n_profiles():
    """roofline.measured: the same-N profile's FETCH_SIZE / WRITE_SIZE bytes per extend launch
    over the run's extend launch time, as GB/s and fractions of the HBM peak; every rank count the driver runs has a
    committed profile of its own N."""
    import json

    import bench

    for n in (1, 2, 4, 8):
        assert (ROOT / "profiles" / bench.pmc_name("C3", n)).exists(), n
        ext = json.loads((ROOT / "profiles" / bench.pmc_name("C3", n)).read_text())["wf_extend_kernel"]
        m = bench.measured_rates("C3", n, 0.02)
        assert m["source"] == f"profiles/{bench.pmc_name('C3', n)}"
        assert m["read_gbs"] == round(ext["fetch_bytes_per_launch"] / 0.02 / 1e9, 1)
        assert m["write_gbs"] == round(ext["write_bytes_per_launch"] / 0.02 / 1e9, 1)
        assert m["read_frac"] == round(m["read_gbs"] / bench.HBM_PEAK_GBS, 4)
    # the N-way profiles are rank 0's shard: their bytes fall with N
    per = [json.loads((ROOT / "profiles" / bench.pmc_name("C3", n)).read_text())["wf_extend_kernel"]["bytes_per_launch"]
           for n in (1, 2, 4, 8)]
    assert per == sorted(per, reverse=True)
    assert bench.measured_rates("no-such-config", 1, 0.02) is None
    assert bench.measured_rates("C3", 3, 0.02) is None  # no profile taken at 3 ranks
    assert bench.measured_rates("C3", 1, 0.0) is None


def test_stdout_to_stderr_catches_native_writes():
    """bench.stdout_to_stderr: output written to fd 1 by native code (gloo's connect messages) goes to stderr, so the
    bench's stdout carries its one JSON line alone."""
    import subprocess
    import sys

    code = ("import os, sys; sys.path.insert(0, %r); import bench\n"
            "with bench.stdout_to_stderr():\n    os.write(1, b'native noise\\n')\n"
            "print('{\"line\": 1}')\n") % str(ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    assert p.stdout == '{"line": 1}\n' and "native noise" in p.stderr
