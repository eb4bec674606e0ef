"""Rank body for tests/test_launch_cpu.py (run by octree_pathtracing_amd.launch.spawn_ranks): joins
the gloo job from the environment the launcher set, checks it, and gathers oracle-rendered tile
shards to rank 0 with the product's distributed.gather_frame; rank 0 saves the frame."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from octree_pathtracing_amd import distributed as D  # noqa: E402


def main():
    out, W, H = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    assert os.environ["MASTER_ADDR"] == "127.0.0.1" and int(os.environ["LOCAL_RANK"]) == rank
    dist.init_process_group("gloo")
    try:
        assert dist.get_world_size() == world and dist.get_rank() == rank
        from oracle import cpu_ref
        from octree_pathtracing_amd import scene as S

        sc, cam, _ = S.make_config("tiny")
        frame = cpu_ref.render(sc, cam, W, H, 1, forward=True, threads=2)[0].reshape(-1, 4)
        stride = D.shard_stride(W, H, world)
        shard = torch.from_numpy(D.extract_shard(frame, W, H, rank, world, stride))
        gbuf = torch.zeros((world * stride, 4), dtype=torch.float32) if rank == 0 else None
        got = D.gather_frame(shard, gbuf, W, H, rank, world, lambda g: D.unshard_host(g.numpy(), W, H, world, stride))
        if rank == 0:
            np.save(out, np.stack([got, frame]))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
