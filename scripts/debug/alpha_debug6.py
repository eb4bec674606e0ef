"""Debug: trace pixel 820 of the alpha world through the megakernel (OCTPT_TRACE_PIXEL build)."""
import sys
sys.path.insert(0, ".")
import torch
from tests.test_gpu_blocks import _alpha_world
from tests.test_gpu_parity import gpu_render
from octree_pathtracing_amd.renderer import HipRenderer

sc, cam, rs = _alpha_world()
rs.max_depth = 2
r = HipRenderer(0, lib_path="build_variants/trace820/liboctpt.so")
a, sa, st = gpu_render(torch, r, sc, cam, rs, megakernel=True)
torch.cuda.synchronize()
print("segs", sa.reshape(-1)[820])
