#!/usr/bin/env python3
"""Headline benchmark: Mrays/s on BASELINE.json's C3 workload (10k spheres, depth-8 octree,
1920x1080, 256 spp, max_depth 5) through the octpt C ABI on MI355X.

A step = one full progressive render of the frame (all 256 passes of every pixel) with the
scene resident in HBM.  With N > 1 GPUs (torchrun, one process per GPU) the frame is split
into 8x8 tiles dealt round-robin to ranks (strong scaling: the frame is fixed), each rank
renders its tiles into a compact buffer and the tiles are gathered to rank 0 over RCCL
(all_gather_into_tensor) and scattered into the frame by octpt_unshard_device.

value = total ray segments (closest-hit queries, all ranks) / wall time of the K timed steps
(max over ranks).  roofline.achieved = algorithmic bytes per render launch /
the launch's average HIP-event duration.  cpu_baseline = the oracle (oracle/cpu_ref.c, a
C port of the reference's CPU TileRenderer) timed on this host on a bounded sample.
"""
from __future__ import annotations

import argparse
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


def algorithmic_bytes(st: dict) -> float:
    """8 B per ESVO iteration (child mask + child word), 16+4 B per sphere test
    (float4 + leaf prim index), 24+4 B per cuboid test, 32 B per shaded hit (GPUMaterial),
    4 B per texel, 16 B per path (running-mean read-modify-write of the F32Color)."""
    return (8.0 * st["esvo_steps"] + 20.0 * st["sphere_tests"] + 28.0 * st["cuboid_tests"]
            + 32.0 * st["shade_events"] + 4.0 * st["texel_reads"] + 16.0 * st["paths"])


def load_traffic(config: str):
    p = ROOT / "profiles" / f"pmc_{config}.json"
    if p.exists():
        try:
            d = json.loads(p.read_text())
            return d.get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def cpu_baseline(sc, cam, rs, seconds: float, threads: int) -> dict:
    """Oracle on the host cores: whole 1 spp passes of the full frame until `seconds` elapse."""
    from oracle import cpu_ref

    acc = None
    segs = 0
    passes = 0
    t0 = time.perf_counter()
    while True:
        acc, _, st = cpu_ref.render(sc, cam, rs.width, rs.height, 1, spp_start=passes, max_depth=rs.max_depth,
                                    seed=rs.seed, threads=threads, accum=acc)
        segs += st["segments"]
        passes += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(segs / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{passes} full-frame pass(es) of the same workload ({rs.width}x{rs.height}, 1 spp each, "
                      f"{segs} segments) in {dt:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None, help="override passes per step (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import HipRenderer, shard_pixels

    sc, cam, rs = S.make_config(args.config)
    if args.spp:
        rs.spp = args.spp
    W, H = rs.width, rs.height
    r = HipRenderer(device=local)
    r.set_scene(sc)
    r.set_camera(cam)
    r.max_depth, r.seed = rs.max_depth, rs.seed
    stride = max(shard_pixels(W, H, i, world) for i in range(world))
    n_local = shard_pixels(W, H, rank, world)
    dev = torch.device("cuda", local)
    accum = torch.zeros((stride, 4), dtype=torch.float32, device=dev)
    accum[:, 3] = 1.0
    gbuf = torch.zeros((world * stride, 4), dtype=torch.float32, device=dev) if world > 1 else None
    frame = torch.zeros((H * W, 4), dtype=torch.float32, device=dev) if (world > 1 and rank == 0) else None
    params = r.params(W, H, 0, rs.spp, rank, world, compact=True)

    def step():
        stream = torch.cuda.current_stream().cuda_stream
        r.render_device(params, accum.data_ptr(), None, stream)
        if world > 1:
            dist.all_gather_into_tensor(gbuf, accum)  # RCCL over xGMI
            if rank == 0:
                r.unshard_device(W, H, world, gbuf.data_ptr(), stride, frame.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
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
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        s = torch.tensor([seg], dtype=torch.float64, device=dev)
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        seg = int(s.item())

    launches = max(st["launches"], 1)
    kernel_s = st["kernel_ms"] / 1e3 / launches
    bytes_per_launch = algorithmic_bytes(st) / launches
    achieved = bytes_per_launch / kernel_s / 1e9 if kernel_s > 0 else 0.0
    traffic = load_traffic(args.config)
    out = {
        "metric": METRIC,
        "value": round(seg / dt / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"{args.config}: {len(sc.spheres)} spheres + {len(sc.cuboids)} cuboids, octree depth "
                        f"{sc.octree.depth}, {W}x{H}, {rs.spp} spp, max_depth {rs.max_depth}, seed {rs.seed}",
            "resolution": [W, H],
            "spp": rs.spp,
            "parallelism": f"tiles{world}" if world > 1 else "single",
            "paths_per_step": W * H * rs.spp,
            "segments_per_step": seg // max(args.steps, 1),
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": "render_kernel",
            "kernel_ms_avg": round(kernel_s * 1e3, 3),
            "algorithmic_bytes_per_launch": int(bytes_per_launch),
        },
        "stats_rank0": {k: v for k, v in st.items() if k != "kernel_ms"},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sc, cam, rs, args.cpu_seconds, args.cpu_threads)
    else:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
