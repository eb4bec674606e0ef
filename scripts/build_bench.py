"""Octree build time: host builder (octpt_build_octree) vs the GPU builder
(octpt_build_octree_device).  Prints the library call's wall time (the device call includes the
primitive upload and the result download) and the GPU time of the build kernels."""
import ctypes as C
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from octree_pathtracing_amd import _lib, scene as S  # noqa: E402
from octree_pathtracing_amd.renderer import HipRenderer  # noqa: E402

r = HipRenderer(0)
lib = _lib.load()


def call(sc, depth, ctx=None, reps=3):
    sph, cub = sc.sphere_structs(), sc.cuboid_structs()
    args = (C.cast(sph, C.c_void_p) if len(sc.spheres) else None, len(sc.spheres),
            C.cast(cub, C.c_void_p) if len(sc.cuboids) else None, len(sc.cuboids), depth)
    best = 1e9
    for _ in range(reps):
        h = C.c_void_p()
        t = time.perf_counter()
        st = lib.octpt_build_octree(*args, C.byref(h)) if ctx is None else \
            lib.octpt_build_octree_device(ctx, *args, C.byref(h))
        best = min(best, time.perf_counter() - t)
        _lib.check(lib, ctx, st)
        lib.octpt_octree_free(h)
    return best


for name in sys.argv[1:] or ["C3", "C4", "C5"]:
    sc, _, _ = S.make_config(name, build=False)
    d = sc._depth
    th = call(sc, d)
    tg = call(sc, d, r._ctx)
    kms = r.stats()["build_ms"]
    n = sc.build_octree(d)
    print(f"{name}: {n.octant_count} octants, {len(n.leaf_first)} leaves, {len(n.leaf_prims)} pairs; host builder "
          f"{th * 1e3:.1f} ms, GPU builder {tg * 1e3:.1f} ms end to end ({th / tg:.1f}x), build kernels "
          f"{kms:.2f} ms ({th * 1e3 / kms:.0f}x)", flush=True)
