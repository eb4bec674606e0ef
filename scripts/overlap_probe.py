"""Experiment: do two wavefront renders on separate streams overlap (extend of one beside shade of the
other)?  Times C3 at SPP spp as one render, then as two concurrent renders of SPP/2 each (two contexts,
two host threads), then the two halves one after the other.  usage: overlap_probe.py [CONFIG] [SPP]"""
import sys
import threading
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch  # noqa: E402

from octree_pathtracing_amd import scene as S  # noqa: E402
from octree_pathtracing_amd.renderer import HipRenderer  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 256
sc, cam, rs = S.make_config(cfg)
W, H = rs.width, rs.height
rr = [HipRenderer(0), HipRenderer(0)]
accs = []
for r in rr:
    r.max_depth, r.seed = rs.max_depth, rs.seed
    r.set_scene(sc)
    r.set_camera(cam)
    a = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda")
    a[:, 3] = 1
    accs.append(a)
streams = [torch.cuda.Stream(), torch.cuda.Stream()]


def render(i, s0, n):
    p = rr[i].params(W, H, s0, n)
    rr[i].render_device(p, accs[i].data_ptr(), None, streams[i].cuda_stream)
    streams[i].synchronize()


for rep in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    render(0, 0, spp)
    one = time.perf_counter() - t
    t = time.perf_counter()
    th = [threading.Thread(target=render, args=(i, i * spp // 2, spp // 2)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    two = time.perf_counter() - t
    t = time.perf_counter()
    render(0, 0, spp // 2)
    render(1, spp // 2, spp // 2)
    seq = time.perf_counter() - t
    print(f"{cfg} {spp} spp: one render {one*1e3:.1f} ms, two concurrent halves {two*1e3:.1f} ms, "
          f"two halves in sequence {seq*1e3:.1f} ms", flush=True)
