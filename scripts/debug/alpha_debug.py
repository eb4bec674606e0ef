"""Debug: GPU vs oracle on the alpha block world (tests/test_gpu_blocks.py::_alpha_world)."""
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from tests.test_gpu_blocks import _alpha_world
from tests.test_gpu_parity import gpu_render, oracle
from octree_pathtracing_amd.renderer import HipRenderer
from oracle import cpu_ref

sc, cam, rs = _alpha_world()
r = HipRenderer(0)
for md in (1, 2, 5):
    rs.max_depth = md
    a, sa, st = gpu_render(torch, r, sc, cam, rs)
    b, sb, rst = oracle(sc, cam, rs, forward=True)
    bad = np.argwhere(sa != sb)
    print("max_depth", md, "seg mismatches", len(bad), bad[:8].tolist(), "gpu blk", st["block_tests"], "ref", rst["block_tests"],
          "steps", st["esvo_steps"], rst["esvo_steps"], flush=True)
# primary rays through pixel centres: intersect
W, H = rs.width, rs.height
dim = max(W, H)
d0 = np.array(cam.direction, np.float32); up = np.array(cam.up, np.float32)
right = np.cross(d0, up).astype(np.float32)
f = np.float32(1.0 / np.tan(cam.fov / 2))
ys, xs = np.mgrid[0:H, 0:W]
xn = ((2 * xs + 1) - W) / dim
yn = ((2 * (H - ys) - 1) - H) / dim
dirs = d0 * f + right * xn[..., None] + up * yn[..., None]
dirs = (dirs / np.linalg.norm(dirs, axis=-1, keepdims=True)).astype(np.float32).reshape(-1, 3)
rays = np.concatenate([np.broadcast_to(np.array(cam.eye, np.float32), dirs.shape), dirs], 1)
r.set_scene(sc)
t, p, n, s = r.intersect(rays)
rt, rp, rn, rsteps = cpu_ref.intersect(sc, rays)
bad = np.nonzero((p != rp) | (s != rsteps) | (t.view(np.uint32) != rt.view(np.uint32)))[0]
print("intersect mismatches", len(bad))
for i in bad[:10]:
    print(i, rays[i].tolist(), "gpu", t[i], hex(p[i]), s[i], n[i].tolist(), "ref", rt[i], hex(rp[i]), rsteps[i], rn[i].tolist())
r.close()
