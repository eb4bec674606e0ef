"""Diagnostic: C3 render time vs spp (prints after every render)."""
import sys, time
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import torch
from octree_pathtracing_amd import scene as S
from octree_pathtracing_amd.renderer import HipRenderer

sc, cam, rs = S.make_config(sys.argv[1] if len(sys.argv) > 1 else "C3")
import os
rs.max_depth = int(os.environ.get("MAXDEPTH", rs.max_depth))  # experiments: primary-only = 1
r = HipRenderer(0)
r.max_depth = rs.max_depth
r.set_scene(sc); r.set_camera(cam)
W, H = rs.width, rs.height
if os.environ.get("TILE_ORDER") == "morton":  # experiments: dealing position -> tile in Morton (Z) order of the tile grid
    import numpy as np
    tx, ty = (W + 7) // 8, (H + 7) // 8
    t = np.arange(tx * ty)
    x, y = t % tx, t // tx
    def part(v):
        v = v.astype(np.uint64) & 0xFFFF
        v = (v | (v << 8)) & 0x00FF00FF
        v = (v | (v << 4)) & 0x0F0F0F0F
        v = (v | (v << 2)) & 0x33333333
        return (v | (v << 1)) & 0x55555555
    r.set_tile_order(W, H, t[np.argsort(part(x) | (part(y) << 1), kind="stable")])
acc = torch.zeros((W * H, 4), dtype=torch.float32, device="cuda"); acc[:, 3] = 1
mega = "--mega" in sys.argv
for spp in [int(x) for x in (a for a in sys.argv[2:] if not a.startswith("--"))] or [4, 16, 64, 256]:
    r.reset_stats()
    r.set_camera(cam)  # every render recomputes the beam table (round 5 caches it for an unchanged camera)
    p = r.params(W, H, 0, spp, megakernel=mega, kernel_timing="--ktime" in sys.argv, preview="--preview" in sys.argv)
    torch.cuda.synchronize(); t = time.perf_counter()
    r.render_device(p, acc.data_ptr(), None, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize(); dt = time.perf_counter() - t
    st = r.stats()
    if st["segments"] == 0:  # stats compiled out (OCTPT_NO_STATS A/B builds)
        print(f"spp {spp}: {dt*1e3:.1f} ms  (no stats)", flush=True)
        continue
    kt = f"  extend {st['extend_ms']:.1f} ms shade {st['shade_ms']:.1f} ms" if st["extend_launches"] else ""
    print(f"spp {spp}: {dt*1e3:.1f} ms  {st['segments']/dt/1e6:.1f} Mrays/s  segs/path {st['segments']/st['paths']:.3f} steps/seg {st['esvo_steps']/st['segments']:.1f}{kt}", flush=True)
