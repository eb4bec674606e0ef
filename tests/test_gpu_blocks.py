"""Block-value leaves on the GPU: the reference's own leaf form -- a leaf payload is a
block id whose box is the leaf cell, at any level (new_octree.rs:534-537, 586, 669, 727), intersected as
octree_traversal.rs:143-214 does -- against the oracle, bit for bit in control flow and within the
render tolerances of tests/test_gpu_parity.py:

- C5's voxel world as block leaves (C5b), and its heightmap as a solid world (C5s-small), plain and
  compacted with the reference's value-equality rule (LOD leaves at levels >= 1);
- the block-model world (blocks-b: block models drawn at their cells, ResourceModel::Quad);
- a tree built the way SectionOctantBuilder does (writer mask encoding, reversed post-order ids),
  uploaded through the reference-scene flattener octpt_scene_from_reference;
- faces with alpha-0 texels (the traversal passes through them), sun sampling, preview, the batch
  closest-hit query and the megakernel (the chunk-tail drain: tests/test_gpu_drain.py)."""
import ctypes as C

import numpy as np
import pytest

from tests.test_blocks_cpu import _reference_scene, block_scene, leaf_levels, random_section
from tests.test_gpu_parity import assert_parity, gpu_render, oracle, rel_err, renderer, torch_cuda  # noqa: F401
from tests import reference_builders as RB

pytestmark = pytest.mark.gpu


def _config(name, res=None, compact=False):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if compact:
        sc.build_octree(sc.octree.depth, compact=True)
    if res:
        rs.width, rs.height, rs.spp = res
    return sc, cam, rs


@pytest.mark.parametrize("name,res,compact", [("blocks-b", None, False), ("C5b", (192, 108, 2), False),
                                              ("C5b-fp", (192, 108, 1), False), ("C5s-small", (192, 108, 2), False),
                                              ("C5s-small", (192, 108, 2), True)])
def test_block_render_parity(torch_cuda, renderer, name, res, compact):
    sc, cam, rs = _config(name, res, compact)
    if compact:
        assert sum(v for k, v in leaf_levels(sc.octree).items() if k >= 1) > 0  # LOD leaves at levels >= 1
    gpu = gpu_render(torch_cuda, renderer, sc, cam, rs)
    ref = oracle(sc, cam, rs, forward=True)
    exact = assert_parity(gpu, ref, name)
    assert gpu[2]["block_tests"] > 0
    assert exact > 0.999, f"{name}: only {exact:.4%} of channels bit-identical"
    rec = oracle(sc, cam, rs, forward=False)
    assert rel_err(gpu[0], rec[0]).max() <= 1e-4


def _section_world(seed=3):
    """A 16^3 section (depth-4 world) built as SectionOctantBuilder builds it, with its camera."""
    from octree_pathtracing_amd import scene as S

    g = random_section(seed)
    sc = block_scene(g, 4, False)  # materials + block table (its own octree is replaced below)
    kind, masks, children = RB.section_octants(g)
    z = np.zeros(0, np.uint32)
    sc.octree = S.Octree(masks, children, 0, 4, z, z.copy(), z.copy())
    cam = S.Camera.look_at((-9.0, 21.0, -13.0), (8.0, 6.0, 8.0))
    return sc, cam, S.RenderSettings(96, 64, 4), masks, children


def test_reference_section_through_flattener(torch_cuda, renderer):
    """The drop-in path end to end: a section tree in the reference's own form (writer mask encoding,
    reversed post-order octant ids, block-value leaves) and the reference's Material / Texture list go
    through octpt_scene_from_reference into octpt_scene_upload, and render as the oracle does."""
    from octree_pathtracing_amd import _lib

    sc, cam, rs, masks, children = _section_world()
    ref, keep = _reference_scene(sc, masks, children, 4)
    n = len(sc.materials)
    mo, to, qo = (_lib.Material * n)(), (_lib.Texture * n)(), (_lib.Quad * 1)()
    desc = _lib.SceneDesc()
    assert renderer._lib.octpt_scene_from_reference(C.byref(ref), mo, to, qo, C.byref(desc)) == _lib.OK
    renderer._check(renderer._lib.octpt_scene_upload(renderer._ctx, C.byref(desc)))
    gpu = gpu_render(torch_cuda, renderer, sc, cam, rs, upload=False)
    assert_parity(gpu, oracle(sc, cam, rs, forward=True), "section")
    # and the same tree uploaded from the Scene directly renders bit-identically
    direct = gpu_render(torch_cuda, renderer, sc, cam, rs)
    assert np.array_equal(direct[0].view(np.uint32), gpu[0].view(np.uint32))


def _alpha_world():
    """Full blocks whose faces hold alpha-0 texels (a glass-pane frame texture, a clear colour texture
    on two faces): the traversal passes through those texels (SingleBlockModel::intersect, C23)."""
    from octree_pathtracing_amd import scene as S

    g = random_section(6, air=0.6, kinds=3)
    sc = block_scene(g, 4, False)
    frame = np.zeros((16, 16), bool)
    frame[[0, 15], :] = frame[:, [0, 15]] = True
    frame[7:9, :] = True
    sc.textures.append(S.Texture.image(S.alpha_tile(3, 354, (200, 225, 235), 10, frame)))
    sc.materials.append(S.Material(texture_index=len(sc.textures) - 1))
    glass = len(sc.materials) - 1
    sc.textures.append(S.Texture.color(255, 255, 255, 0))
    sc.materials.append(S.Material(texture_index=len(sc.textures) - 1))
    clear = len(sc.materials) - 1
    sc.blocks[1] = glass
    sc.blocks[2, [1, 4]] = clear
    sc.build_octree(4)
    cam = S.Camera.look_at((-9.0, 21.0, -13.0), (8.0, 6.0, 8.0))
    return sc, cam, S.RenderSettings(96, 64, 4)


def test_alpha_faces_parity(torch_cuda, renderer):
    sc, cam, rs = _alpha_world()
    gpu = gpu_render(torch_cuda, renderer, sc, cam, rs)
    assert_parity(gpu, oracle(sc, cam, rs, forward=True), "alpha")
    # the transparent texels matter: the same world with opaque faces renders differently
    rs.max_depth = 1
    a = gpu_render(torch_cuda, renderer, sc, cam, rs)
    sc.blocks[1] = sc.blocks[3]
    b = gpu_render(torch_cuda, renderer, sc, cam, rs)
    assert a[2]["esvo_steps"] != b[2]["esvo_steps"]


@pytest.mark.parametrize("variant", ["fast", "hq_sss"])
def test_block_sun_sampling_parity(torch_cuda, renderer, variant):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = _config("C5s-small", (160, 90, 2), compact=True)
    S.with_sun_variant(sc, variant)
    assert_parity(gpu_render(torch_cuda, renderer, sc, cam, rs), oracle(sc, cam, rs, forward=True), variant)


@pytest.mark.parametrize("name,res,compact", [("blocks-b", None, False), ("C5b", (320, 180, 1), False),
                                              ("C5s-small", (320, 180, 1), True)])
def test_block_preview_parity(torch_cuda, renderer, name, res, compact):
    sc, cam, rs = _config(name, res, compact)
    acc, segs, st = gpu_render(torch_cuda, renderer, sc, cam, rs, preview=True)
    racc, rsegs, rst = oracle(sc, cam, rs, preview=True)
    assert np.array_equal(segs, rsegs)
    assert st["segments"] == rst["segments"] and st["esvo_steps"] == rst["esvo_steps"]
    assert np.array_equal(acc, racc)


@pytest.mark.parametrize("name,compact", [("C5s-small", True), ("C5s-small", False), ("blocks-b", False),
                                          ("section", False)])
def test_block_intersect_parity(renderer, name, compact):
    from oracle import cpu_ref

    if name == "section":
        sc = _section_world()[0]
        lo, hi = -4.0, 20.0
    else:
        sc = _config(name, compact=compact)[0]
        lo, hi = (0.0, 180.0) if name.startswith("C5") else (0.0, 32.0)
    rng = np.random.default_rng(11)
    n = 20000
    o = rng.uniform(lo, hi, (n, 3)).astype(np.float32)
    d = rng.normal(size=(n, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], 1)
    renderer.set_scene(sc)
    t, prim, nrm, steps = renderer.intersect(rays)
    rt, rprim, rnrm, rsteps = cpu_ref.intersect(sc, rays)
    assert np.array_equal(prim, rprim) and np.array_equal(steps, rsteps)
    assert np.array_equal(t.view(np.uint32), rt.view(np.uint32)) and np.array_equal(nrm, rnrm)
    assert (prim != 0xFFFFFFFF).sum() > n // 20


@pytest.mark.parametrize("name,res", [("blocks-b", None), ("C5s-small", (160, 90, 2))])
def test_block_megakernel_equals_wavefront(torch_cuda, renderer, name, res):
    sc, cam, rs = _config(name, res, compact=name == "C5s-small")
    a = gpu_render(torch_cuda, renderer, sc, cam, rs)
    b = gpu_render(torch_cuda, renderer, sc, cam, rs, megakernel=True)
    assert np.array_equal(a[1], b[1]) and rel_err(a[0], b[0]).max() <= 1e-5
    assert a[2]["esvo_steps"] == b[2]["esvo_steps"] and a[2]["block_tests"] == b[2]["block_tests"]


def test_c5b_fullframe_oracle(torch_cuda, renderer):
    """C5 as block leaves at the full 3840 x 2160, 1 spp, against the oracle over the whole frame."""
    sc, cam, rs = _config("C5b")
    rs.spp = 1
    gpu = gpu_render(torch_cuda, renderer, sc, cam, rs)
    exact = assert_parity(gpu, oracle(sc, cam, rs, forward=True, threads=16), "C5b")
    assert gpu[2]["block_tests"] > 0 and exact > 0.999


def test_block_upload_validation(renderer):
    from octree_pathtracing_amd import _lib

    sc, cam, rs = _config("blocks-b")
    desc, keep = sc.to_desc()
    lib = renderer._lib
    assert lib.octpt_scene_upload(renderer._ctx, C.byref(desc)) == _lib.OK
    saved = desc.block_count
    desc.block_count = 1  # leaf payloads beyond the block table
    assert lib.octpt_scene_upload(renderer._ctx, C.byref(desc)) == _lib.ERR_INVALID_ARG
    assert b"block" in lib.octpt_last_error(renderer._ctx)
    desc.block_count = saved
    sph = (_lib.Sphere * 1)()
    desc.spheres, desc.sphere_count = C.cast(sph, C.c_void_p), 1  # primitives beside block leaves
    assert lib.octpt_scene_upload(renderer._ctx, C.byref(desc)) == _lib.ERR_INVALID_ARG
    desc.spheres, desc.sphere_count = None, 0
    assert lib.octpt_scene_build_device(renderer._ctx, C.byref(desc), 0) == _lib.ERR_INVALID_ARG
