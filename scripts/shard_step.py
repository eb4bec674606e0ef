#!/usr/bin/env python3
"""One step of rank K's work in an N-way tile split, in one process: the shard render bench.py's rank K runs
(OCTPT_RENDER_SHARD_COMPACT over its 8x8 tiles, its chunk and pool sized for its own items), without the
gather.  Used under rocprofv3 --pmc to profile a shard of the same N as the N-rank bench line quotes
(profiles/pmc_<config>_n<N>.json), and prints the shard's extend figures as one JSON line.
Usage: python scripts/shard_step.py [--config C3] [--n 8] [--k 0] [--spp S] [--warmup 0]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--k", type=int, default=0)
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=0)
    args = ap.parse_args()
    assert 0 <= args.k < args.n
    import torch

    import bench
    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import HipRenderer, shard_pixels

    sc, cam, rs = S.make_config(args.config)
    if args.spp:
        rs.spp = args.spp
    W, H = rs.width, rs.height
    with HipRenderer(device=0) as r:
        r.set_scene(sc)
        r.set_camera(cam)
        r.max_depth, r.seed = rs.max_depth, rs.seed
        acc = torch.zeros((shard_pixels(W, H, args.k, args.n), 4), dtype=torch.float32, device="cuda")
        p = r.params(W, H, 0, rs.spp, args.k, args.n, compact=True, kernel_timing=True)
        stream = torch.cuda.current_stream().cuda_stream
        for _ in range(args.warmup):
            r.render_device(p, acc.data_ptr(), None, stream)
        torch.cuda.synchronize()
        r.reset_stats()
        r.set_camera(cam)  # the beam table recomputed (an unchanged camera would reuse it)
        t0 = time.perf_counter()
        r.render_device(p, acc.data_ptr(), None, stream)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        st = r.stats()
    n_ext = max(st["extend_launches"], 1)
    roof = bench.roofline_over_ranks([{"bytes": bench.extend_bytes(st), "ext_ms": st["extend_ms"],
                                       "launches": st["extend_launches"]}])
    print(json.dumps({"config": args.config, "shard": [args.k, args.n], "spp": rs.spp, "ms": round(dt * 1e3, 3),
                      "mrays_s": round(st["segments"] / dt / 1e6, 2), "segments": st["segments"],
                      "extend_launches": st["extend_launches"],
                      "extend_ms_avg": round(st["extend_ms"] / n_ext, 4),
                      "algorithmic_bytes_per_launch": int(bench.extend_bytes(st) / n_ext),
                      "achieved": roof["achieved"], "frac": roof["frac"]}), flush=True)


if __name__ == "__main__":
    main()
