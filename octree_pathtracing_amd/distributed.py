"""Multi-GPU tile sharding of the render: one process per GPU.

The frame's 8x8 pixel tiles are dealt round-robin, tile t -> rank t % N (or, with a tile order set --
octpt_set_tile_order, octpt_balance_tiles -- the tile at dealing position t); rank k renders its tiles
into a compact buffer (OCTPT_RENDER_SHARD_COMPACT: tile-major, 64 pixels per tile, row-major inside
the tile -- the kernels' item_pixel mapping, octpt_kernels.hip) of `stride` pixels (the largest
shard), the compact buffers are gathered to rank 0 (RCCL over xGMI on the GPUs, gloo in the CPU tests)
and rank 0 scatters them back into the frame (octpt_unshard_device on the GPU, unshard_host here).
Per-pixel RNG streams are keyed by pixel and sample, never by rank, so a sharded render equals the
unsharded one bit for bit.
"""
from __future__ import annotations

import numpy as np

TILE = 8


def tiles_xy(W: int, H: int):
    return (W + TILE - 1) // TILE, (H + TILE - 1) // TILE


def dealt_tiles(W: int, H: int, k: int, N: int, order=None) -> np.ndarray:
    """Frame tiles of shard k in its local order: dealing positions k + u * N, through the tile order
    (octpt_set_tile_order: order[s] = the frame tile at position s) when one is set."""
    tx, ty = tiles_xy(W, H)
    s = np.arange(k, tx * ty, N)
    return s if order is None else np.asarray(order)[s]


def shard_tile_count(W: int, H: int, k: int, N: int) -> int:
    tx, ty = tiles_xy(W, H)
    tiles = tx * ty
    return len(range(k, tiles, N))


def shard_stride(W: int, H: int, N: int) -> int:
    """Pixels per compact shard buffer: the largest shard (shard 0)."""
    return shard_tile_count(W, H, 0, N) * TILE * TILE


def shard_layout(W: int, H: int, k: int, N: int, order=None) -> np.ndarray:
    """Frame pixel index (y * W + x) of every compact slot of shard k; -1 where the tile overhangs
    the image (those slots hold zero radiance)."""
    tx, _ = tiles_xy(W, H)
    t = dealt_tiles(W, H, k, N, order)
    w = np.arange(64)
    x = (t[:, None] % tx) * TILE + (w[None, :] & 7)
    y = (t[:, None] // tx) * TILE + (w[None, :] >> 3)
    idx = np.where((x < W) & (y < H), y * W + x, -1)
    return idx.reshape(-1)


def extract_shard(frame: np.ndarray, W: int, H: int, k: int, N: int, stride: int | None = None,
                  order=None) -> np.ndarray:
    """Compact shard k of a full frame [H*W, 4] (what rank k's render produces)."""
    stride = stride or shard_stride(W, H, N)
    lay = shard_layout(W, H, k, N, order)
    out = np.zeros((stride, frame.shape[-1]), frame.dtype)
    ok = lay >= 0
    out[: len(lay)][ok] = frame.reshape(-1, frame.shape[-1])[lay[ok]]
    return out


def unshard_host(shards: np.ndarray, W: int, H: int, N: int, stride: int, order=None) -> np.ndarray:
    """Host mirror of unshard_kernel: gathered shards [N * stride, 4] -> frame [H * W, 4]."""
    frame = np.zeros((W * H, shards.shape[-1]), shards.dtype)
    for k in range(N):
        lay = shard_layout(W, H, k, N, order)
        ok = lay >= 0
        frame[lay[ok]] = shards[k * stride: k * stride + len(lay)][ok]
    return frame


def gather_frame(accum, gbuf, W: int, H: int, rank: int, world: int, unshard):
    """Gather the ranks' compact shards (tensors [stride, 4]) to rank 0 into gbuf [world * stride, 4]
    (rank 0 only; None elsewhere) and let rank 0 scatter them into the frame with `unshard(gbuf)`.
    One dist.gather: on RCCL a group of point-to-point transfers into rank 0 over xGMI (each rank
    sends its 1/N of the frame once, N - 1 shards arrive), not an all-gather that would hand every
    rank the whole frame.  Returns unshard's result on rank 0, None elsewhere."""
    import torch.distributed as dist

    if world == 1:
        return unshard(accum) if rank == 0 else None
    stride = accum.shape[0]
    parts = [gbuf[i * stride:(i + 1) * stride] for i in range(world)] if rank == 0 else None
    dist.gather(accum, gather_list=parts, dst=0)
    return unshard(gbuf) if rank == 0 else None


def gather_rank_values(values, world: int, device="cpu") -> list:
    """Every rank's list of floats (the same length on every rank) to every rank, in rank order: one
    all_gather of a float64 vector (bench.py's per-rank extend bytes / times for the N-GPU roofline)."""
    import torch
    import torch.distributed as dist

    mine = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if world == 1:
        return [mine.tolist()]
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    return [p.cpu().tolist() for p in parts]
