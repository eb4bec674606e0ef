"""The C ABI driven from a plain C host (tools/capi_host.c, built by __graft_entry__.build()): no Python in the
render path, as the Rust shim of INTEGRATION.md §3 would drive it.  The C program builds a sphere scene with the
library's host builder, uploads it, renders a progressive frame synchronously then asynchronously, and runs a
closest-hit batch; the same scene through the Python bindings must give the same frame and hits bit for bit, and
the oracle the same per-frame statistics and radiance within the parity tolerance.  It then runs the shim's own
set_scene sequence: a block-value tree in the reference writer's encoding
through octpt_scene_from_reference and octpt_scene_upload, a FrameInFlight render, and a two-entry context
(octpt_create_multi over [0, 0]); test_c_host_reference_sequence checks that frame."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

from tests.test_gpu_parity import REL_TOL_FORWARD, gpu_render, rel_err, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]
W, H, SPP_SYNC, SPP_ASYNC, NSPH, NRAYS = 96, 64, 3, 2, 24, 256


def capi_scene():
    """tools/capi_host.c's scene and camera, built through the Python scene types."""
    from octree_pathtracing_amd import scene as S

    sc = S.Scene()
    i = np.arange(NSPH)
    sp = np.zeros((NSPH, 4), np.float32)
    sp[:, 0] = 4.0 + (i * 7) % 24 + 0.25 * (i % 3)
    sp[:, 1] = 6.0 + (i * 5) % 13
    sp[:, 2] = 6.0 + (i * 11) % 20 + 0.5 * (i % 2)
    sp[:, 3] = 1.0 + 0.125 * (i % 4)
    sc.spheres = sp
    sc.sphere_material = (1 + i % 2).astype(np.uint32)
    sc.textures = [S.Texture(), S.Texture.color(200, 60, 40), S.Texture.color(230, 230, 235)]
    sc.materials = [S.air_material(), S.Material(texture_index=1),
                    S.Material(metalness=1.0, roughness=0.1, texture_index=2)]
    sc.build_octree(5)
    f = lambda v: float(np.float32(v))  # noqa: E731
    cam = S.Camera(eye=(16.0, 22.0, -6.0), direction=(0.0, f(-0.4472136), f(0.8944272)),
                   up=(0.0, f(0.8944272), f(0.4472136)))
    return sc, cam


def _run_host(tmp_path, *extra):
    exe = ROOT / "tools" / "capi_host"
    assert exe.exists(), "build it with __graft_entry__.build()"
    out = tmp_path / "capi.bin"
    p = subprocess.run([str(exe), str(out), *map(str, extra)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    return out


class _Reader:
    def __init__(self, raw):
        self.raw, self.o = raw, 0

    def take(self, dtype, n):
        a = np.frombuffer(self.raw, dtype, n, self.o)
        self.o += a.nbytes
        return a


def test_c_host_reference_sequence(torch_cuda, renderer, tmp_path):
    """The Rust shim's set_scene of INTEGRATION.md §3, in C: a block-value world in the reference writer's form
    (octants as bit i + 8 alone, children before parents, LOD leaves), the reference's Material list, the
    flattener, the upload, render_async / poll / wait / release, and the same frame through octpt_create_multi
    over [0, 0].  Both C frames must equal each other and the frame the Python bindings render from the same
    arrays through the same flattener, bit for bit, and the oracle within the parity tolerance."""
    import ctypes as C

    from octree_pathtracing_amd import _lib
    from octree_pathtracing_amd import scene as S
    from oracle import cpu_ref
    from tests.test_blocks_cpu import _reference_scene, leaf_levels

    ref_out = tmp_path / "ref.bin"
    _run_host(tmp_path, ref_out)
    r = _Reader(ref_out.read_bytes())
    n_oct, root, depth, n_blk, n_mat, iw, ih, spp = (int(v) for v in r.take(np.uint32, 8))
    masks = r.take(np.uint32, n_oct).astype(np.uint16)
    children = r.take(np.uint32, 8 * n_oct).reshape(n_oct, 8).copy()
    blocks = r.take(np.uint32, 6 * n_blk).reshape(n_blk, 6).copy()
    mats, texs = [], []
    for i in range(n_mat):
        ior, spec, emit, rough, metal = (float(v) for v in r.take(np.float32, 5))
        flags, kind = (int(v) for v in r.take(np.uint32, 2))
        col = tuple(int(v) for v in r.take(np.uint8, 4))
        mats.append(S.Material(ior=ior, specular=spec, emittance=emit, roughness=rough, metalness=metal,
                               texture_index=i, flags=flags))
        texs.append((kind, col))
    img = r.take(np.uint8, iw * ih * 4).reshape(ih, iw, 4).copy()
    eye, d, up = (tuple(float(v) for v in r.take(np.float32, 3)) for _ in range(3))
    fov = float(r.take(np.float32, 1)[0])
    acc1 = r.take(np.float32, W * H * 4).reshape(H, W, 4)
    acc2 = r.take(np.float32, W * H * 4).reshape(H, W, 4)
    r.take(np.uint8, W * H * 4)
    paths1, segs1, blk1, paths2, segs2, blk2 = (int(v) for v in r.take(np.uint64, 6))
    assert r.o == len(r.raw)

    # the tree is in the writer's form, with LOD leaves above level 0, and its root is the last octant
    assert root == n_oct - 1 and any(((m >> i) & 0x101) == 0x100 for m in masks for i in range(8))
    sc = S.Scene()
    sc.materials = mats
    sc.textures = [S.Texture.image(img) if k == _lib.TEXTURE_IMAGE else S.Texture.color(*c) for k, c in texs]
    sc.blocks = blocks
    sc.block_model = np.full(n_blk, _lib.MODEL_NONE, np.uint32)
    z = np.zeros(0, np.uint32)
    sc.octree = S.Octree(masks, children, root, depth, z, z.copy(), z.copy())
    assert sum(v for k, v in leaf_levels(sc.octree).items() if k >= 1) > 0
    cam = S.Camera(eye=eye, direction=d, up=up, fov=fov)

    # the C host's two contexts agree, and every pass of every pixel was rendered
    assert np.array_equal(acc1.view(np.uint32), acc2.view(np.uint32)), "octpt_create_multi([0, 0]) != one context"
    assert paths1 == paths2 == W * H * spp and segs1 == segs2 and blk1 == blk2 > 0
    # the same arrays through the same flattener from Python
    rsc, keep = _reference_scene(sc, masks, children, depth, root=root)
    mo, to, qo = (_lib.Material * n_mat)(), (_lib.Texture * n_mat)(), (_lib.Quad * 1)()
    desc = _lib.SceneDesc()
    assert renderer._lib.octpt_scene_from_reference(C.byref(rsc), mo, to, qo, C.byref(desc)) == _lib.OK
    renderer._check(renderer._lib.octpt_scene_upload(renderer._ctx, C.byref(desc)))
    rs = S.RenderSettings(W, H, spp, seed=1)
    py = gpu_render(torch_cuda, renderer, sc, cam, rs, upload=False)
    assert np.array_equal(py[0].view(np.uint32), acc1.view(np.uint32)), "C host frame != Python frame"
    assert py[2]["segments"] == segs1
    # and the oracle on the reference-form tree
    racc, _, rst = cpu_ref.render(sc, cam, W, H, spp, seed=1, forward=True)
    assert rst["segments"] == segs1
    assert rel_err(acc1, racc).max() <= REL_TOL_FORWARD


def test_c_host_equals_python_and_oracle(torch_cuda, renderer, tmp_path):
    from octree_pathtracing_amd import scene as S
    from oracle import cpu_ref

    exe = ROOT / "tools" / "capi_host"
    assert exe.exists(), "build it with __graft_entry__.build()"
    out = tmp_path / "capi.bin"
    p = subprocess.run([str(exe), str(out)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    raw = out.read_bytes()
    o = 0

    def take(dtype, n):
        nonlocal o
        a = np.frombuffer(raw, dtype, n, o)
        o += a.nbytes
        return a

    accum = take(np.float32, 4 * W * H).reshape(H, W, 4)
    take(np.uint8, 4 * W * H)
    rays = take(np.float32, 6 * NRAYS).reshape(NRAYS, 6)
    t, prim, steps = take(np.float32, NRAYS), take(np.uint32, NRAYS), take(np.uint32, NRAYS)
    paths, segments, _ = take(np.uint64, 3)
    assert o == len(raw)

    sc, cam = capi_scene()
    rs = S.RenderSettings(W, H, SPP_SYNC, seed=1)
    first = gpu_render(torch_cuda, renderer, sc, cam, rs)
    rs.spp = SPP_ASYNC
    second = gpu_render(torch_cuda, renderer, sc, cam, rs, spp_start=SPP_SYNC, accum=first[0])
    assert np.array_equal(second[0].view(np.uint32), accum.view(np.uint32)), "C host frame != Python frame"
    assert paths == W * H * (SPP_SYNC + SPP_ASYNC)
    assert segments == first[2]["segments"] + second[2]["segments"]
    pt, pprim, _, psteps = renderer.intersect(rays)
    assert np.array_equal(pprim, prim) and np.array_equal(psteps, steps)
    assert np.array_equal(pt.view(np.uint32), t.view(np.uint32))
    # the oracle: the same five passes, and Scene::hit on the same rays
    racc, _, rst = cpu_ref.render(sc, cam, W, H, SPP_SYNC + SPP_ASYNC, seed=1, forward=True)
    assert rst["segments"] == segments
    assert rel_err(accum, racc).max() <= REL_TOL_FORWARD
    rt, rprim, _, rsteps = cpu_ref.intersect(sc, rays)
    hit = rprim != 0xFFFFFFFF
    assert np.array_equal(rprim, prim) and np.array_equal(rsteps, steps) and hit.sum() > 20
    assert np.array_equal(rt[hit], t[hit])
