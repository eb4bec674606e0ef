"""Debug: megakernel / wavefront / drain-off vs oracle on the alpha block world."""
import os, sys
sys.path.insert(0, ".")
import numpy as np
import torch
from tests.test_gpu_blocks import _alpha_world
from tests.test_gpu_parity import gpu_render, oracle
from octree_pathtracing_amd.renderer import HipRenderer

sc, cam, rs = _alpha_world()
rs.max_depth = 2
b, sb, rst = oracle(sc, cam, rs, forward=True)
r = HipRenderer(0)
for mk in (False, True):
    a, sa, st = gpu_render(torch, r, sc, cam, rs, megakernel=mk)
    print("megakernel" if mk else "wavefront", "seg mismatches", int((sa != sb).sum()), "blk", st["block_tests"], rst["block_tests"],
          "drain segs", st["drain"]["segments"], flush=True)
r.close()
os.environ["OCTPT_DRAIN_RAYS"] = "0"
r = HipRenderer(0)
a, sa, st = gpu_render(torch, r, sc, cam, rs)
print("no drain seg mismatches", int((sa != sb).sum()), "blk", st["block_tests"], flush=True)
os.environ["OCTPT_POOL"] = "64"
r2 = HipRenderer(0)
a, sa, st = gpu_render(torch, r2, sc, cam, rs)
print("pool 64 seg mismatches", int((sa != sb).sum()), "blk", st["block_tests"], flush=True)
