#!/usr/bin/env python3
"""Headline benchmark: Mrays/s on BASELINE.json's C3 workload (10k spheres, depth-8 octree,
1920x1080, 256 spp, max_depth 5) through the octpt C ABI on MI355X.

A step = one full progressive render of the frame (all 256 passes of every pixel) with the
scene resident in HBM.  With N > 1 GPUs (torchrun, one process per GPU) the frame is split
into 8x8 tiles dealt round-robin to ranks (strong scaling: the frame is fixed), each rank
renders its tiles into a compact buffer and the tiles are gathered to rank 0 over RCCL
(dist.gather) and scattered into the frame by octpt_unshard_device.  `--gpus N` started without
torchrun spawns the N ranks itself (octree_pathtracing_amd/launch.py) before anything touches the
GPU; under torchrun WORLD_SIZE must equal N.

value = total ray segments (closest-hit queries, all ranks) / wall time of the K timed steps
(max over ranks).  roofline: the dominant kernel is wf_extend_kernel (octree traversal +
primitive tests, ~90 % of GPU time); achieved = its algorithmic bytes per launch
/ its average launch duration, both measured live: every extend / shade launch of the timed
steps is bracketed by HIP events on the render stream (OCTPT_RENDER_KERNEL_TIMING).  traffic =
the L2-to-fabric bytes per extend launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes
committed in profiles/pmc_<config>.json (traffic_source names the file and the FETCH_SIZE factor
calibrated by tools/fetch_calib.hip).  cpu_baseline = the oracle (oracle/cpu_ref.c, a C port of
the reference's CPU TileRenderer) built -O3 -march=native on this host and timed on a bounded
sample with the host's CPU share of threads (model, nproc and flags recorded).
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "Mrays/sec at 1920×1080×256spp; achieved HBM GB/s vs roofline at 1/2/4/8 GPUs"


def extend_share(st: dict) -> dict:
    """The counters of the extend launches: the totals minus the chunk-tail drain kernel's share
    (octpt_stats.drain; the drain is timed apart, rocprof lists it as wf_drain_kernel)."""
    d = st.get("drain", {})
    return {k: st.get(k, 0) - d.get(k, 0) for k in ("segments", "esvo_steps", "sphere_tests", "cuboid_tests",
                                                      "block_tests", "issued_bytes")}


def extend_bytes(st: dict) -> float:
    """SURVEY.md §8(d) for wf_extend_kernel: 8 B per ESVO iteration (one node record:
    child mask + child payload; reference iterations, the folded ones included), 16 + 4 B per sphere
    test (centre/radius float4 + leaf prim index), 24 + 4 B per cuboid test (min/max + index); a
    block-value leaf (C23) is the node record alone.  The wavefront's own queue traffic
    (extend_queue_bytes) is not in §8(d) and is reported beside it.  Drain work excluded."""
    e = extend_share(st)
    return 8.0 * e["esvo_steps"] + 20.0 * e["sphere_tests"] + 28.0 * e["cuboid_tests"]


def extend_queue_bytes(st: dict) -> float:
    """The wavefront's queue traffic in extend: 32-B ray record read + 8-B hit record write per segment."""
    return 40.0 * extend_share(st)["segments"]


def lean_state(sc, st: dict) -> bool:
    """Whether the renders ran with the lean 24-B path state: no emitter (with emitters
    on), no sun sampling, the pool holding the chunk, OCTPT_LEAN not 0 -- octpt_scene_upload's lean_scene
    and enqueue_wavefront's per-chunk rule."""
    emissive = sc.emitters_enabled and any(m.emittance > 5e-8 for m in sc.materials)
    return (not emissive and not sc.strategy.sun_sampling and st["pool_slots"] >= st["chunk_items"]
            and os.environ.get("OCTPT_LEAN", "") != "0")


def shade_bytes(st: dict, lean: bool = False, lds_tables: bool = False) -> float:
    """DESIGN.md §8, wf_shade_kernel's global-memory bytes per segment: ray record 32 + hit 8 + path state read, path
    state + ray record 32 written (the path state 40 B, or 24 B in the lean state); per shaded hit 16 (sphere or box
    record) + 4 (material id) + 48 (material record, unless the scene's material tables sit in LDS: lds_tables,
    shade_lds_tables); 4 B per texel; 16 B per finished path (colour record).  Until round 4 the 48 B of an
    LDS-resident material record were counted too."""
    per_seg = 40.0 + 2.0 * (24.0 if lean else 40.0) + 32.0
    per_event = 20.0 + (0.0 if lds_tables else 48.0)
    return (per_seg * st["segments"] + per_event * st["shade_events"] + 4.0 * st["texel_reads"] + 16.0 * st["paths"])


def shade_lds_tables(sc) -> bool:
    """Whether shade reads the material / texture tables from LDS (octpt_kernels.hip shade_lds_tables: <= 128 of each)."""
    return len(sc.materials) <= 128 and len(sc.textures) <= 128


def pmc_name(config: str, world: int = 1) -> str:
    """The committed PMC profile a line of `config` at `world` ranks may quote: profiles/pmc_<config>.json for
    one GPU, profiles/pmc_<config>_n<N>.json (rank 0's shard of an N-way split, scripts/shard_step.py) else."""
    return f"pmc_{config}.json" if world == 1 else f"pmc_{config}_n{world}.json"


def load_pmc(config: str, world: int = 1):
    """(the wf_extend_kernel record, source description) of the profile pmc_name(config, world) names, or
    (None, reason): a line at N ranks never quotes a profile taken at another N."""
    name = pmc_name(config, world)
    p = ROOT / "profiles" / name
    if p.exists():
        try:
            d = json.loads(p.read_text())
            return d.get("wf_extend_kernel", {}), f"profiles/{name}: {d.get('correction', '')}"
        except Exception as e:
            return None, f"profiles/{name} unreadable ({type(e).__name__})"
    return None, f"no PMC profile of {config} at {world} rank(s) (profiles/{name})"


def load_traffic(config: str, world: int = 1):
    """(bytes per extend launch, source description, L2 hit rate) from the profile pmc_name(config, world)
    names, or (None, reason, None)."""
    ext, src = load_pmc(config, world)
    if ext is None:
        return None, src, None
    return ext.get("bytes_per_launch"), src, ext.get("l2_hit_rate")


def measured_rates(config: str, world: int, ext_s: float):
    """BASELINE.json's "achieved HBM GB/s" as rocprof measures it: the same-N profile's FETCH_SIZE (read) and
    WRITE_SIZE (write) bytes per wf_extend_kernel launch (L2-to-fabric requests, Infinity-Cache hits included,
    so an upper bound of HBM bytes; rank 0's shard at N > 1) over this run's mean extend launch duration on the
    same rank, each as a fraction of one GPU's HBM peak.  None without a same-N profile."""
    ext, src = load_pmc(config, world)
    if not ext or ext_s <= 0 or "fetch_bytes_per_launch" not in ext:
        return None
    rd, wr = ext["fetch_bytes_per_launch"] / ext_s / 1e9, ext["write_bytes_per_launch"] / ext_s / 1e9
    return {"read_gbs": round(rd, 1), "read_frac": round(rd / HBM_PEAK_GBS, 4),
            "write_gbs": round(wr, 1), "write_frac": round(wr / HBM_PEAK_GBS, 4),
            "total_gbs": round(rd + wr, 1), "total_frac": round((rd + wr) / HBM_PEAK_GBS, 4),
            "l2_hit_rate": ext.get("l2_hit_rate"), "launches_profiled": ext.get("launches"),
            "source": src.split(":")[0],
            "basis": "rocprofv3 FETCH_SIZE / WRITE_SIZE bytes per extend launch of the same-N profile (rank 0's "
                     "shard at N > 1) / this run's mean extend launch duration on rank 0 (HIP events); fabric "
                     "bytes, Infinity-Cache hits included: an upper bound of HBM traffic"}


def roofline_over_ranks(ranks: list) -> dict:
    """The extend roofline over N ranks (BASELINE.json's "achieved HBM GB/s vs roofline at 1/2/4/8 GPUs").
    `ranks`: one dict per rank with `bytes` (algorithmic extend bytes of the timed steps, drain excluded),
    `ext_ms` (the summed durations of its extend launches) and `launches`.  Rank r achieves
    bytes_r / ext_ms_r; `achieved` is the per-GPU mean, `aggregate_gbs` = sum of the ranks' bytes / the
    slowest rank's extend time, against `aggregate_peak` = N x the one-GPU peak; frac_min / frac_max give
    the spread over ranks."""
    per = []
    for r in ranks:
        t = r["ext_ms"] / 1e3
        per.append(r["bytes"] / t / 1e9 if t > 0 else 0.0)
    n = len(ranks)
    tmax = max(r["ext_ms"] for r in ranks) / 1e3
    agg = sum(r["bytes"] for r in ranks) / tmax / 1e9 if tmax > 0 else 0.0
    mean = sum(per) / n
    return {"achieved": round(mean, 1), "frac": round(mean / HBM_PEAK_GBS, 4),
            "aggregate_gbs": round(agg, 1), "aggregate_peak": HBM_PEAK_GBS * n,
            "aggregate_frac": round(agg / (HBM_PEAK_GBS * n), 4),
            "frac_min": round(min(per) / HBM_PEAK_GBS, 4), "frac_max": round(max(per) / HBM_PEAK_GBS, 4),
            "per_rank": [{"rank": i, "achieved": round(a, 1), "bytes": int(r["bytes"]), "ext_ms": round(r["ext_ms"], 3),
                          "launches": int(r["launches"])} for i, (a, r) in enumerate(zip(per, ranks))]}


def host_cpu() -> dict:
    """The host the CPU baseline runs on: model, logical CPUs, the affinity mask and the thread
    share used (the box's OMP_NUM_THREADS share when set: a GPU box's nproc shows the whole machine)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    share = os.environ.get("OMP_NUM_THREADS")
    threads = min(aff, int(share)) if share and share.isdigit() and int(share) > 0 else aff
    return {"model": model, "nproc": os.cpu_count(), "affinity": aff, "threads": threads}


def native_oracle():
    """Build the oracle -O3 -march=native for this host (oracle/Makefile `native`, into oracle/_native/;
    the x86-64-v2 build stays the parity checker) and return (path, flags), or the portable build."""
    import subprocess

    try:
        # -B: always for this host (a library built on another machine's -march=native may not run here)
        subprocess.run(["make", "-s", "-B", "-C", str(ROOT / "oracle"), "native"], check=True, capture_output=True,
                       timeout=180)
        return ROOT / "oracle" / "_native" / "libcpu_ref_native.so", "-O3 -march=native -ffp-contract=off"
    except Exception:
        return ROOT / "oracle" / "libcpu_ref.so", "-O2 -march=x86-64-v2 -ffp-contract=off (native build failed)"


def _cpu_rate(sc, cam, rs, seconds: float, threads: int, rows=None):
    """Oracle Mrays/s on `threads` threads: 1-spp passes of the frame (or of `rows`) until `seconds` elapse."""
    from oracle import cpu_ref

    acc = None
    segs = passes = 0
    t0 = time.perf_counter()
    while True:
        acc, _, st = cpu_ref.render(sc, cam, rs.width, rs.height, 1, spp_start=passes, max_depth=rs.max_depth,
                                    seed=rs.seed, threads=threads, accum=acc, rows=rows)
        segs += st["segments"]
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return segs / dt / 1e6, passes, segs, dt


def cpu_baseline(sc, cam, rs, seconds: float, threads: int | None) -> dict:
    """The oracle (oracle/cpu_ref.c, -O3 -march=native) on the host: whole 1-spp passes of the full
    frame on the box's CPU share (OMP_NUM_THREADS; the pool's rule for worker pools), and
    one thread on a band of rows for the per-core rate.  SURVEY §8(d) asks for all host cores: that
    figure is the per-core rate times the affinity cores, a linear upper bound stated as such."""
    from oracle import cpu_ref

    host = host_cpu()
    n = threads or host["threads"]
    lib_path, flags = native_oracle()
    cpu_ref.load(lib_path)
    rate, passes, segs, dt = _cpu_rate(sc, cam, rs, seconds, n)
    band = (rs.height // 2 - 32, rs.height // 2 + 32)  # the frame's middle 64 rows, one thread
    rate1, passes1, segs1, dt1 = _cpu_rate(sc, cam, rs, max(seconds / 3.0, 2.0), 1, rows=band)
    return {"value": round(rate, 3), "unit": "Mrays/s", "cores": n, "kind": "port",
            "sample": f"{passes} full-frame pass(es) of the same workload ({rs.width}x{rs.height}, 1 spp each, "
                      f"{segs} segments) in {dt:.1f} s on {n} threads; 1 thread: {passes1} pass(es) of rows "
                      f"{band[0]}-{band[1]} ({segs1} segments) in {dt1:.1f} s",
            "per_core": round(rate1, 4),
            "all_cores_linear": {"value": round(rate1 * host["affinity"], 2), "cores": host["affinity"],
                                 "basis": "per-core rate x affinity cores (linear upper bound, not measured)"},
            "cpu_model": host["model"], "nproc": host["nproc"], "affinity": host["affinity"], "build": flags}


def issued_probe(sc, cam, rs, dev_idx: int, ext_s: float):
    """One render of the same step through the OCTPT_COUNT_ISSUED diagnostic library:
    the bytes extend actually issues per launch (node slots of the lanes that load one, primitives,
    quads, alpha texels) and the roofline fraction they give over the timed library's launch time."""
    lib = ROOT / "octree_pathtracing_amd" / "lib" / "liboctpt_issued.so"
    if not lib.exists():
        return None
    import torch
    from octree_pathtracing_amd.renderer import HipRenderer, balance_tiles, shard_pixels

    r = HipRenderer(device=dev_idx, lib_path=str(lib))
    try:
        r.set_scene(sc)
        r.set_camera(cam)
        r.max_depth, r.seed = rs.max_depth, rs.seed
        W, H = rs.width, rs.height
        acc = torch.zeros((shard_pixels(W, H, 0, 1), 4), dtype=torch.float32, device=torch.device("cuda", dev_idx))
        acc[:, 3] = 1.0
        r.render_device(r.params(W, H, 0, rs.spp, 0, 1, compact=True, kernel_timing=True), acc.data_ptr(), None,
                        torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        st = r.stats()
    finally:
        r.close()
    n = max(st["extend_launches"], 1)
    e = extend_share(st)
    per_launch = e["issued_bytes"] / n
    achieved = per_launch / ext_s / 1e9 if ext_s > 0 else 0.0
    return {"bytes_per_launch": int(per_launch), "achieved": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "launches": st["extend_launches"],
            "basis": "liboctpt_issued.so (-DOCTPT_COUNT_ISSUED): every load extend issues, summed by the kernel; "
                     "one render of the same step, divided by the timed library's mean extend launch time"}


def capi_devices(spec: str, n_visible: int) -> list:
    """--capi-devices: "N" = the first N visible devices (repeating device ids when fewer are visible, as on
    a one-GPU box), or an explicit comma-separated list of HIP device ids."""
    if "," in spec:
        return [int(x) for x in spec.split(",")]
    return [i % max(n_visible, 1) for i in range(int(spec))]


def capi_multi_measure(config: str, devices, steps: int, warmup: int, spp=None, compact: bool = False,
                       timeout: float = 600.0) -> dict:
    """The multi-device path a Rust host calls (octpt_create_multi): one process, one context over
    `devices`, whole frames through octpt_render_device into a frame buffer on devices[0] (tiles dealt over the
    entries, gathered with peer copies inside liboctpt) -- `bench.py --capi-devices` run as a child process, so that
    a failure of this extra leg (the first distinct-device peer copies on a node) is reported in the line instead
    of ending the N-rank bench that runs it.  Whole-job Mrays/s over the timed steps."""
    import subprocess

    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    cmd = [sys.executable, str(Path(__file__).resolve()), "--config", config, "--capi-devices",
           ",".join(str(d) for d in devices), "--steps", str(steps), "--warmup", str(warmup), "--no-cpu-baseline",
           "--no-issued", *(["--spp", str(spp)] if spp else []), *(["--compact"] if compact else [])]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    if p.returncode != 0 or not lines:
        return {"error": f"exit {p.returncode}: {(p.stderr or p.stdout)[-600:]}", "devices": list(devices)}
    d = json.loads(lines[-1])
    return {"value": d["value"], "unit": d["unit"], "devices": d["config"]["capi_devices"],
            "ms_per_step": d["ms_per_step"], "steps": d["steps"], "segments": d["config"]["segments_per_step"],
            "path": "octpt_create_multi + octpt_render_device (one child process, peer-copy gather inside liboctpt)"}


def balance_deal(r, segbuf, n_local: int, W: int, H: int, rank: int, world: int, cdev, balance_tiles) -> str:
    """The N-rank tile deal of the timed steps: every rank's per-tile segment counts of the last
    warmup step (its compact shard, 64 pixels per tile, dealt round robin) go to every rank, and each rank sets
    the same order octpt_balance_tiles derives from them -- the previous frame's cost, as a progressive renderer
    has it.  Rank 0's unshard follows the order (the same context)."""
    from octree_pathtracing_amd.distributed import dealt_tiles, gather_rank_values, tiles_xy

    mine = segbuf[:n_local].cpu().numpy().view(np.uint32).reshape(-1, 64).sum(1, dtype=np.int64)
    most = max(len(dealt_tiles(W, H, k, world)) for k in range(world))
    rows = gather_rank_values(np.pad(mine, (0, most - len(mine))).tolist(), world, cdev)
    tx, ty = tiles_xy(W, H)
    img = np.zeros(W * H, np.uint32)  # each tile's cost at its first pixel: balance_tiles sums per tile
    for k in range(world):
        t = dealt_tiles(W, H, k, world)
        img[(t // tx) * 8 * W + (t % tx) * 8] = np.asarray(rows[k][:len(t)], np.float64).astype(np.uint32)
    r.set_tile_order(W, H, balance_tiles(W, H, world, img))
    return "balanced: octpt_balance_tiles over the warmup step's per-tile segment counts"


@contextlib.contextmanager
def stdout_to_stderr():
    """fd 1 redirected to fd 2 for the block (output printed by native code, which sys.stdout does not see)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def scene_contents(sc) -> str:
    if sc.blocks is not None:  # block-value leaves
        return f"{len(sc.cells)} voxel cells as block-value leaves ({len(sc.blocks)} block kinds)"
    return f"{len(sc.spheres)} spheres + {len(sc.cuboids)} cuboids"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None, help="override passes per step (default: the config's)")
    ap.add_argument("--compact", action="store_true",
                    help="build the octree with OCTPT_BUILD_COMPACT (is_compactable merge, DESIGN.md C22)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: the host's CPU share (host_cpu)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-issued", action="store_true", help="skip the issued-bytes probe (diagnostic library)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: host-staged gather (rehearses N ranks on fewer GPUs); nccl = RCCL over xGMI")
    ap.add_argument("--dump-frame", default=None, help="rank 0 saves the gathered frame (.npy) after the last step")
    ap.add_argument("--capi-devices", default=None,
                    help="one process, one multi-device context (octpt_create_multi) over N devices or a list of "
                         "HIP ids: the C-ABI path a Rust host calls (DESIGN.md §9); ids repeat on a one-GPU box")
    ap.add_argument("--balance", action="store_true",
                    help="with N > 1 ranks, time the steps under the tile order octpt_balance_tiles derives from the "
                         "warmup step's per-tile segment counts instead of the round-robin deal (DESIGN.md §9: "
                         "measured equal on C3 / C5b, so round robin stays the default)")
    ap.add_argument("--no-capi-multi", action="store_true",
                    help="with N > 1 ranks, skip rank 0's extra measurement of the same frame through one "
                         "multi-device context over the N devices (after the timed steps; the other ranks wait on a "
                         "gloo group, so no RCCL kernel sits on the GPUs it renders on)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU without torchrun: spawn the ranks before anything touches the GPU
        from octree_pathtracing_amd.launch import spawn_ranks

        sys.exit(spawn_ranks(args.gpus, [str(Path(__file__).resolve()), *sys.argv[1:]]))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}", file=sys.stderr)
        sys.exit(2)
    n_dev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > n_dev:
        print(f"bench.py: {world} ranks over RCCL need {world} GPUs, {n_dev} visible", file=sys.stderr)
        sys.exit(2)
    dev_idx = local % max(n_dev, 1)
    torch.cuda.set_device(dev_idx)
    host_group = None
    if world > 1:
        # gloo prints "[Gloo] Rank r is connected to ..." on stdout from C++ while it connects: stdout carries the
        # bench's one JSON line, so the connects run with fd 1 pointed at stderr
        with stdout_to_stderr():
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
            else:
                dist.init_process_group("gloo")
            # rank 0's extra legs after the timed steps are waited for on this host-side group (below)
            host_group = dist.new_group(backend="gloo")
        assert dist.get_world_size() == args.gpus

    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.distributed import gather_frame, gather_rank_values
    from octree_pathtracing_amd.renderer import HipRenderer, balance_tiles, shard_pixels

    sc, cam, rs = S.make_config(args.config, build=not args.compact)
    if args.compact:
        sc.build_octree(sc._depth, compact=True)
    spp_default = rs.spp
    if args.spp:
        rs.spp = args.spp
    # a committed PMC profile is of the config's own frame: a run at another spp (other launches) quotes none
    pmc_ok = rs.spp == spp_default and not args.compact
    W, H = rs.width, rs.height
    multi = capi_devices(args.capi_devices, n_dev) if (args.capi_devices and world == 1) else None
    r = HipRenderer(devices=multi) if multi else HipRenderer(device=dev_idx)
    r.set_scene(sc)
    r.set_camera(cam)
    r.max_depth, r.seed = rs.max_depth, rs.seed
    stride = max(shard_pixels(W, H, i, world) for i in range(world))
    n_local = shard_pixels(W, H, rank, world)
    dev = torch.device("cuda", dev_idx)
    host_staged = world > 1 and args.dist_backend == "gloo"
    accum = torch.zeros((stride, 4), dtype=torch.float32, device=dev)
    accum[:, 3] = 1.0
    gdev = "cpu" if host_staged else dev
    gbuf = torch.zeros((world * stride, 4), dtype=torch.float32, device=gdev) if (world > 1 and rank == 0) else None
    gbuf_dev = torch.zeros((world * stride, 4), dtype=torch.float32, device=dev) if (host_staged and rank == 0) else None
    frame = torch.zeros((H * W, 4), dtype=torch.float32, device=dev) if (world > 1 and rank == 0) else None
    params = r.params(W, H, 0, rs.spp, rank, world, compact=True, kernel_timing=True)
    if multi:  # the whole frame in image order on devices[0]: the multi-device context gathers it itself
        accum = torch.zeros((W * H, 4), dtype=torch.float32, device=dev)
        accum[:, 3] = 1.0
        params = r.params(W, H, 0, rs.spp, kernel_timing=True)

    def unshard(g):
        stream = torch.cuda.current_stream().cuda_stream
        if host_staged:
            gbuf_dev.copy_(g)
            g = gbuf_dev
        r.unshard_device(W, H, world, g.data_ptr(), stride, frame.data_ptr(), stream)

    balance = world > 1 and args.balance and args.warmup > 0
    segbuf = torch.zeros(stride, dtype=torch.int32, device=dev) if balance else None

    def step(seg=None):
        stream = torch.cuda.current_stream().cuda_stream
        # the camera set again: the beam table is recomputed every step (a render with an unchanged camera would
        # reuse it, as a progressive renderer's next frame does), so a step carries the whole frame's work
        r.set_camera(cam)
        r.render_device(params, accum.data_ptr(), seg.data_ptr() if seg is not None else None, stream)
        if world > 1:  # gather to rank 0 (RCCL over xGMI), then the unshard kernel on rank 0
            src = accum.cpu() if host_staged else accum
            gather_frame(src, gbuf, W, H, rank, world, unshard)

    for i in range(args.warmup):
        step(segbuf if i == args.warmup - 1 else None)
    torch.cuda.synchronize()
    deal = "round robin"
    if balance:  # the warmup step's per-tile segments, all ranks' to every rank, then one order everywhere
        deal = balance_deal(r, segbuf, n_local, W, H, rank, world, gdev, balance_tiles)
    r.reset_stats()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    st = r.stats()
    seg = st["segments"]
    mine = [dt, float(seg), extend_bytes(st), st["extend_ms"], float(st["extend_launches"])]
    if world > 1:  # every rank's figures to every rank (collectives on the backend's device; gloo: host)
        rows = gather_rank_values(mine, world, gdev)
        dt = max(r[0] for r in rows)
        seg = int(sum(r[1] for r in rows))
    else:
        rows = [mine]
    over = roofline_over_ranks([{"bytes": r[2], "ext_ms": r[3], "launches": r[4]} for r in rows])

    n_ext = max(st["extend_launches"], 1)
    ext_s = st["extend_ms"] / 1e3 / n_ext
    bytes_per_launch = extend_bytes(st) / n_ext  # drain work excluded (extend_share)
    n_sh = max(st["shade_launches"], 1)
    sh_s = st["shade_ms"] / 1e3 / n_sh
    lean = lean_state(sc, st)
    sh_bytes = shade_bytes(st, lean, shade_lds_tables(sc)) / n_sh
    traffic, traffic_src, l2_hit = load_traffic(args.config, world) if pmc_ok else \
        (None, f"the committed profiles are of {args.config}'s own frame ({spp_default} spp, full octree)", None)
    out = {
        "metric": METRIC,
        "value": round(seg / dt / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "msamples_per_s": round(W * H * rs.spp * args.steps / dt / 1e6, 2),  # paths/s
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: {scene_contents(sc)}, octree depth {sc.octree.depth} "
                        f"({sc.octree.octant_count} octants{', compacted' if args.compact else ''}), {W}x{H}, "
                        f"{rs.spp} spp, max_depth {rs.max_depth}, seed {rs.seed}",
            "resolution": [W, H],
            "spp": rs.spp,
            "parallelism": ((f"tiles{world}" + ("-gloo" if host_staged else "")) if world > 1
                            else f"capi-multi{len(multi)}" if multi else "single"),
            "paths_per_step": W * H * rs.spp,
            "tile_deal": deal if world > 1 else None,
            "segments_per_step": seg // max(args.steps, 1),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": over["achieved"],
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": over["frac"],
            "traffic": traffic,
            "traffic_source": traffic_src,
            "l2_hit_rate": l2_hit,
            "kernel": "wf_extend_kernel",
            # rank 0's launches (at N > 1 the per-rank figures are in `ranks`, the aggregate beside)
            "launches": st["extend_launches"],
            "kernel_ms_avg": round(ext_s * 1e3, 4),
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
            "bytes_basis": "SURVEY.md §8(d): 8 B x ESVO iterations + 20 B x sphere tests + 28 B x cuboid tests "
                           "(block-value leaves: the node record only); drain kernel excluded",
            "queue_bytes_per_launch": int(extend_queue_bytes(st) / n_ext),
            "share_of_gpu_time": round(st["extend_ms"] / max(st["extend_ms"] + st["shade_ms"], 1e-9), 3),
            "shade": {"kernel": "wf_shade_kernel", "launches": st["shade_launches"],
                      "kernel_ms_avg": round(sh_s * 1e3, 4), "algorithmic_bytes_per_launch": int(sh_bytes),
                      "achieved": round(sh_bytes / sh_s / 1e9, 1) if sh_s > 0 else 0.0,
                      "path_state_bytes": 24 if lean else 40,
                      "bytes_basis": "global-memory bytes of the shade model (DESIGN.md §8): queue + path state + "
                                     "primitive records + texels + colour records; LDS-resident material tables "
                                     "excluded; latency-bound, not at its bandwidth"},
        },
        "stats_rank0": {k: v for k, v in st.items() if k != "kernel_ms"},
    }
    if world > 1:  # achieved = the per-GPU mean; the whole job's extend GB/s against N x the peak
        out["roofline"].update({k: over[k] for k in ("aggregate_gbs", "aggregate_peak", "aggregate_frac", "frac_min",
                                                     "frac_max")})
        out["roofline"]["ranks"] = over["per_rank"]
        out["roofline"]["achieved_basis"] = "mean over ranks of each rank's extend bytes / its extend time"
    if multi:
        out["config"]["capi_devices"] = multi
    out["roofline"]["measured"] = measured_rates(args.config, world, ext_s) if pmc_ok else None
    # After the timed steps and the gather, rank 0 alone runs the extra legs (the C-ABI multi-device frame, the
    # CPU baseline) while the other ranks wait on a gloo group: a wait on the RCCL group would leave an RCCL kernel
    # resident on the GPUs the multi-device leg renders on.
    if world > 1 and not args.no_capi_multi:
        # the same frame through the C-ABI path a Rust host calls: one process (rank 0), one multi-device
        # context over the N devices, tiles gathered inside liboctpt.  (gloo rehearsals of N ranks
        # on fewer GPUs repeat device ids, as the ranks do)
        if rank == 0:
            try:
                devs = [i % max(n_dev, 1) for i in range(world)]
                out["capi_multi"] = capi_multi_measure(args.config, devs, args.steps, args.warmup, args.spp,
                                                       args.compact)
            except Exception as e:  # reported, never fatal to the bench line
                out["capi_multi"] = {"error": f"{type(e).__name__}: {e}"}
        dist.barrier(group=host_group)
    if rank == 0 and world == 1 and not args.no_issued and not multi:
        out["roofline"]["issued"] = issued_probe(sc, cam, rs, dev_idx, ext_s)
    # the reference's CPU path timed in the same run next to the N-GPU figure (north_star), on rank 0 only
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sc, cam, rs, args.cpu_seconds, args.cpu_threads)
        out["cpu_baseline"]["gpu_over_cpu"] = round(out["value"] / max(out["cpu_baseline"]["value"], 1e-9), 1)
    else:
        out["cpu_baseline"] = None
    if world > 1:
        dist.barrier(group=host_group)
    if rank == 0:
        print(json.dumps(out), flush=True)
        if args.dump_frame:  # the frame in image order (a single rank's buffer is tile-major too)
            if multi:
                frame = accum
            elif world == 1:
                frame = torch.zeros((H * W, 4), dtype=torch.float32, device=dev)
                r.unshard_device(W, H, 1, accum.data_ptr(), stride, frame.data_ptr(),
                                 torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            np.save(args.dump_frame, frame.cpu().numpy())
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
