"""Debug: determinism of the alpha block world render, and the zeroed-stack variant."""
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
for lib in (None, "build_variants/zerostack/liboctpt.so"):
    r = HipRenderer(0, lib_path=lib)
    for k in range(3):
        a, sa, st = gpu_render(torch, r, sc, cam, rs)
        print(lib, k, "seg mismatches", int((sa != sb).sum()), "blk", st["block_tests"], rst["block_tests"], flush=True)
    for k in range(2):
        a, sa, st = gpu_render(torch, r, sc, cam, rs, megakernel=True)
        print(lib, "mk", k, "seg mismatches", int((sa != sb).sum()), "blk", st["block_tests"], flush=True)
    r.close()
