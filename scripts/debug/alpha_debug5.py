"""Debug: find the alpha-world pixels where the megakernel differs from the oracle."""
import sys
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
a, sa, st = gpu_render(torch, r, sc, cam, rs, megakernel=True)
bad = np.argwhere(sa != sb)
print("mk mismatches", len(bad), [(int(y) * rs.width + int(x), int(sa[y, x]), int(sb[y, x])) for y, x in bad[:10]])
