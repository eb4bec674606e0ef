"""Device-resident scene build (octpt_scene_build_device): the GPU builder's arrays are
packed into the device node slots in place.  The resulting scene must be the one octpt_scene_upload
makes from the host builder's octree: renders bit-identical in radiance, per-pixel segment counts and
ESVO / primitive-test totals, closest-hit queries identical in t, primitive, normal and steps."""
import time

import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

STAT_KEYS = ("segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads")


def _rays(sc, n, seed):
    rng = np.random.default_rng(seed)
    w = float(1 << sc.octree.depth)
    o = rng.uniform(-0.1 * w, 1.1 * w, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return np.concatenate([o, d], 1).astype(np.float32)


@pytest.mark.parametrize("name,res,compact", [("tiny", None, False), ("tiny", None, True),
                                              ("C2", (160, 90, 4), False), ("C3", (192, 108, 2), False),
                                              ("C3", (192, 108, 2), True), ("C4", (128, 72, 2), False),
                                              ("C4", (128, 72, 2), True), ("C5", (192, 108, 1), False),
                                              ("C5", (192, 108, 1), True), ("blocks", None, False)])
def test_scene_build_device_equals_upload(torch_cuda, renderer, name, res, compact):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name, build=False)
    if res:
        rs.width, rs.height, rs.spp = res
    depth = sc._depth
    sc.build_octree(depth, compact=compact)
    a = gpu_render(torch_cuda, renderer, sc, cam, rs)
    hit_a = renderer.intersect(_rays(sc, 4096, 7))
    renderer.set_scene_built(sc, depth, compact=compact)
    b = gpu_render(torch_cuda, renderer, sc, cam, rs, upload=False)
    hit_b = renderer.intersect(_rays(sc, 4096, 7))
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "radiance"
    assert np.array_equal(a[1], b[1]), "segment counts"
    for k in STAT_KEYS:
        assert a[2][k] == b[2][k], k
    for x, y in zip(hit_a, hit_b):
        assert np.array_equal(np.asarray(x).view(np.uint32), np.asarray(y).view(np.uint32))


def test_scene_build_device_empty_and_errors(torch_cuda, renderer):
    from octree_pathtracing_amd import _lib
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("C1-as-is")  # no primitives: a childless root, sky + sun only
    a = gpu_render(torch_cuda, renderer, sc, cam, rs)
    renderer.set_scene_built(S.Scene(materials=sc.materials, textures=sc.textures), sc.octree.depth)
    b = gpu_render(torch_cuda, renderer, sc, cam, rs, upload=False)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    # a desc carrying an octree is refused (the device build makes it)
    sc2, _, _ = S.make_config("tiny")
    desc, keep = sc2.to_desc()
    lib = _lib.load()
    import ctypes as C

    assert lib.octpt_scene_build_device(renderer._ctx, C.byref(desc), 0) == _lib.ERR_INVALID_ARG
    assert lib.octpt_scene_build_device(renderer._ctx, C.byref(desc), 0x100) == _lib.ERR_INVALID_ARG
    desc2, keep2 = sc2.to_desc(octree=False, depth=0)
    assert lib.octpt_scene_build_device(renderer._ctx, C.byref(desc2), 0) == _lib.ERR_INVALID_ARG
    big = S.Scene()
    big.cuboids = np.array([[0, 0, 0, 2047.5, 2047.5, 2047.5]], np.float32)  # 2^33 cells
    big.cuboid_material = np.zeros((1, 6), np.uint32)
    with pytest.raises(_lib.OctptError) as e:
        renderer.set_scene_built(big, 11)
    assert e.value.status == _lib.ERR_OOM


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_scene_build_device_timing(torch_cuda, renderer, name):
    """End-to-end scene set-up on the device (primitive upload + build + slot packing + tables)
    against the host path (GPU build, download, octpt_scene_upload).  Recorded, not asserted beyond
    the device path being no slower."""
    from octree_pathtracing_amd import scene as S

    sc, _, _ = S.make_config(name, build=False)
    depth = sc._depth
    renderer.set_scene_built(sc, depth)  # warm: scratch and code objects
    t0 = time.perf_counter()
    renderer.set_scene_built(sc, depth)
    torch_cuda.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    sc.build_octree(depth, renderer=renderer)
    renderer.set_scene(sc)
    torch_cuda.cuda.synchronize()
    host_ms = (time.perf_counter() - t0) * 1e3
    print(f"\n{name}: device-resident scene set-up {dev_ms:.1f} ms, device build + host round trip {host_ms:.1f} ms")
    assert dev_ms < host_ms * 1.2
