"""The N > 1 path on the CPU: tile shards of a render all-gathered over gloo (world size 2 and 3,
127.0.0.1 rendezvous) and scattered back into the frame must equal the unsharded render bit for
bit, with shard sizes equal to liboctpt's octpt_shard_pixels.  The radiance comes from the oracle
(test infrastructure); the layout, gather and unshard are the product's (distributed.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from octree_pathtracing_amd import distributed as D


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _frame(W, H):
    from oracle import cpu_ref
    from octree_pathtracing_amd import scene as S

    sc, cam, _ = S.make_config("tiny")
    acc, _, _ = cpu_ref.render(sc, cam, W, H, 2, forward=True, threads=2)
    return acc.reshape(-1, 4)


def _worker(rank, world, port, W, H, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from octree_pathtracing_amd import _lib

        frame = _frame(W, H)  # every rank renders the same deterministic frame (pixel-keyed RNG)
        stride = D.shard_stride(W, H, world)
        assert _lib.load().octpt_shard_pixels(W, H, rank, world) == D.shard_tile_count(W, H, rank, world) * 64
        shard = torch.from_numpy(D.extract_shard(frame, W, H, rank, world, stride))
        gbuf = torch.zeros((world * stride, 4), dtype=torch.float32) if rank == 0 else None
        out = D.gather_frame(shard, gbuf, W, H, rank, world,
                             lambda g: D.unshard_host(g.numpy(), W, H, world, stride))
        if rank == 0:
            q.put(bool(np.array_equal(out, frame)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H", [(2, 40, 24), (3, 37, 19)])
def test_gloo_tile_gather_equals_frame(world, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("W,H,N", [(64, 48, 2), (70, 45, 3), (9, 17, 4), (1920, 1080, 8)])
def test_layout_is_a_partition(W, H, N):
    seen = np.concatenate([D.shard_layout(W, H, k, N) for k in range(N)])
    seen = seen[seen >= 0]
    assert len(seen) == W * H and np.array_equal(np.sort(seen), np.arange(W * H))
    stride = D.shard_stride(W, H, N)
    rng = np.random.default_rng(0)
    frame = rng.random((W * H, 4), dtype=np.float32)
    shards = np.concatenate([D.extract_shard(frame, W, H, k, N, stride) for k in range(N)])
    assert np.array_equal(D.unshard_host(shards, W, H, N, stride), frame)


def _values_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = D.gather_rank_values([rank, 10.0 * rank + 0.5, 1e12 + rank], world)
        q.put((rank, rows))
    finally:
        dist.destroy_process_group()


def test_gloo_gather_rank_values():
    """bench.py's per-rank figures (extend bytes / time) reach every rank in rank order (world size 2)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_values_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    want = [[float(r), 10.0 * r + 0.5, 1e12 + r] for r in range(world)]
    got = [q.get(timeout=5) for _ in range(world)]
    assert all(rows == want for _, rows in got)


@pytest.mark.parametrize("W,H,N", [(64, 48, 2), (70, 45, 3), (1920, 1080, 8), (3840, 2160, 8)])
def test_balance_tiles(W, H, N):
    """octpt_balance_tiles (host, no GPU): a permutation of the frame's tiles in dealing order; shard k keeps its
    round-robin number of tiles, in image order; on a skewed per-pixel cost map the most loaded shard carries
    less than under the round-robin deal, and never more than the mean plus the costliest tile."""
    from octree_pathtracing_amd.renderer import balance_tiles

    tx, ty = D.tiles_xy(W, H)
    T = tx * ty
    rng = np.random.default_rng(W + H + N)
    yy, xx = np.mgrid[0:H, 0:W]
    seg = (rng.integers(0, 4, (H, W)) + 8 * ((xx // 8) % N == 1) + 5 * (yy * 3 < H)).astype(np.uint32)
    order = balance_tiles(W, H, N, seg)
    assert order.dtype == np.uint32 and np.array_equal(np.sort(order), np.arange(T))
    tile_cost = np.zeros(T, np.int64)
    np.add.at(tile_cost, ((yy // 8) * tx + xx // 8).reshape(-1), seg.reshape(-1).astype(np.int64))
    rr, bal = [], []
    for k in range(N):
        mine = D.dealt_tiles(W, H, k, N, order)
        assert len(mine) == D.shard_tile_count(W, H, k, N) and np.all(np.diff(mine) > 0)
        rr.append(tile_cost[D.dealt_tiles(W, H, k, N)].sum())
        bal.append(tile_cost[mine].sum())
    assert sum(bal) == sum(rr) == tile_cost.sum()
    assert max(bal) <= max(rr) and max(bal) <= tile_cost.sum() / N + tile_cost.max()
    if N > 2:
        assert max(bal) < max(rr)
    # the layout helpers follow the order: shards of a frame scatter back to it
    stride = D.shard_stride(W, H, N)
    frame = rng.random((W * H, 4), dtype=np.float32)
    shards = np.concatenate([D.extract_shard(frame, W, H, k, N, stride, order) for k in range(N)])
    assert np.array_equal(D.unshard_host(shards, W, H, N, stride, order), frame)
    assert not np.array_equal(D.unshard_host(shards, W, H, N, stride), frame)


def test_balance_tiles_arguments():
    import ctypes as C

    from octree_pathtracing_amd import _lib

    lib = _lib.load()
    seg = (C.c_uint32 * 64)()
    order = (C.c_uint32 * 1)()
    assert lib.octpt_balance_tiles(8, 8, 0, seg, order) == _lib.ERR_INVALID_ARG
    assert lib.octpt_balance_tiles(8, 8, 2, None, order) == _lib.ERR_INVALID_ARG
    assert lib.octpt_balance_tiles(0, 8, 2, seg, order) == _lib.ERR_INVALID_ARG
    assert lib.octpt_balance_tiles(8, 8, 2, seg, order) == 0 and order[0] == 0
    assert lib.octpt_set_tile_order(None, 8, 8, order) == _lib.ERR_INVALID_ARG
