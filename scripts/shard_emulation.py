#!/usr/bin/env python3
"""Strong-scaling rehearsal on one GPU: time every shard of an N-way tile split of the bench
frame (C3, 1920x1080x256 by default) one after the other.  max over shards ~ the N-GPU step
time without the RCCL gather; sum/ max = the load-balance ceiling of the speed-up.
--balance: each N-way split under the tile order octpt_balance_tiles derives from the one-GPU frame's per-pixel
segment counts, instead of the round-robin deal.
Usage: python scripts/shard_emulation.py [--config C3] [--spp 256] [--ns 1 2 4 8] [--balance]"""
import argparse
import json

import numpy as np
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--ns", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--balance", action="store_true")
    ap.add_argument("--lanes", type=int, default=1,
                    help="render each shard through one context of this many entries on device 0 (octpt_create_multi: "
                         "the shard's tiles split again over concurrent wavefronts on the one GPU)")
    args = ap.parse_args()
    import torch
    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import HipRenderer, balance_tiles, shard_pixels

    sc, cam, rs = S.make_config(args.config)
    if args.spp:
        rs.spp = args.spp
    W, H = rs.width, rs.height
    r = HipRenderer(devices=[0] * args.lanes) if args.lanes > 1 else HipRenderer(device=0)
    r.set_scene(sc)
    r.set_camera(cam)
    r.max_depth, r.seed = rs.max_depth, rs.seed
    out = {"config": args.config, "spp": rs.spp, "deal": "balanced" if args.balance else "round robin", "lanes": args.lanes,
           "runs": {}}
    stream = torch.cuda.current_stream().cuda_stream
    seg_full = None
    if args.balance:  # the one-GPU frame's per-pixel segment counts, the cost the balanced deal evens out
        acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
        seg = torch.zeros(W * H, dtype=torch.int32, device="cuda")
        r.render_device(r.params(W, H, 0, rs.spp), acc.data_ptr(), seg.data_ptr(), stream)
        torch.cuda.synchronize()
        seg_full = seg.cpu().numpy().view(np.uint32)
        del acc, seg
    for n in args.ns:
        r.set_tile_order(W, H, balance_tiles(W, H, n, seg_full) if args.balance else None)
        times, segs = [], []
        for k in range(n):
            acc = torch.zeros((shard_pixels(W, H, k, n), 4), dtype=torch.float32, device="cuda")
            p = r.params(W, H, 0, rs.spp, k, n, compact=True)
            r.render_device(p, acc.data_ptr(), None, stream)  # warm (allocations)
            torch.cuda.synchronize()
            acc.zero_()
            r.reset_stats()
            r.set_camera(cam)  # the beam table recomputed (an unchanged camera would reuse it)
            t0 = time.perf_counter()
            r.render_device(p, acc.data_ptr(), None, stream)
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
            segs.append(r.stats()["segments"])
        t1 = out["runs"].get("1", {}).get("max_ms")
        mx = max(times) * 1e3
        out["runs"][str(n)] = {"max_ms": round(mx, 2), "min_ms": round(min(times) * 1e3, 2),
                               "mean_ms": round(sum(times) / n * 1e3, 2),
                               "seg_imbalance": round(max(segs) / (sum(segs) / n), 4),
                               "speedup_vs_1": round(t1 / mx, 3) if t1 else None}
        print(json.dumps({n: out["runs"][str(n)]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
