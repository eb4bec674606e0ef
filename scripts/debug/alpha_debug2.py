"""Debug: GPU vs oracle closest hits on the alpha block world from every side."""
import sys
sys.path.insert(0, ".")
import numpy as np
from tests.test_gpu_blocks import _alpha_world
from octree_pathtracing_amd.renderer import HipRenderer
from oracle import cpu_ref

sc, cam, rs = _alpha_world()
r = HipRenderer(0)
r.set_scene(sc)
rng = np.random.default_rng(1)
n = 20000
o = rng.uniform(-6, 22, (n, 3)).astype(np.float32)
tgt = rng.uniform(1, 15, (n, 3)).astype(np.float32)
d = tgt - o
d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
rays = np.concatenate([o, d], 1)
t, p, nn, s = r.intersect(rays)
rt, rp, rn, rsteps = cpu_ref.intersect(sc, rays)
bad = np.nonzero((p != rp) | (s != rsteps) | (t.view(np.uint32) != rt.view(np.uint32)))[0]
print("intersect mismatches", len(bad), "of", n, "hits", (p != 0xFFFFFFFF).sum())
for i in bad[:12]:
    print(i, rays[i].tolist(), "gpu", t[i], hex(p[i]), s[i], nn[i].tolist(), "ref", rt[i], hex(rp[i]), rsteps[i], rn[i].tolist())
r.close()
