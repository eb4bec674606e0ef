"""The hit-record check: liboctpt_checkhits.so (-DOCTPT_CHECK_HITS) starts every extend
step's primitive hit with sentinel fields and counts each hit record a field of which shade reads -- a
sphere's root flag, a cuboid's face flags and t, a block leaf's t and (u, v) -- still holds the sentinel: a
field the path that produced the hit did not write, or a codegen merge that let a lane keep the value it
entered the step with, the defect that left block-leaf (u, v) stale in round 3.  Every instance is rendered
(spheres, boxes, block models, block values with alpha-0 faces and models, the drain) and must count none,
with frames equal to the product library's."""
import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def checked(torch_cuda):
    import __graft_entry__ as g
    from octree_pathtracing_amd.renderer import HipRenderer

    assert g.LIB_CHECKHITS.exists(), "build it with __graft_entry__.build()"
    r = HipRenderer(device=0, lib_path=str(g.LIB_CHECKHITS))
    yield r
    r.close()


@pytest.mark.parametrize("name,res", [("tiny", None), ("C3", (320, 180, 4)), ("C4", (256, 144, 2)),
                                      ("C5", (256, 144, 2)), ("C5b", (256, 144, 2)), ("blocks", None),
                                      ("blocks-b", None), ("C5s-small", (160, 90, 2)), ("alpha", None)])
def test_no_unwritten_hit_fields(torch_cuda, renderer, checked, name, res):
    from octree_pathtracing_amd import scene as S

    if name == "alpha":
        from tests.test_gpu_blocks import _alpha_world

        sc, cam, rs = _alpha_world()
    else:
        sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    a = gpu_render(torch_cuda, checked, sc, cam, rs)
    assert a[2]["hit_check_failures"] == 0, (name, a[2]["hit_check_failures"])
    b = gpu_render(torch_cuda, renderer, sc, cam, rs)
    assert b[2]["hit_check_failures"] == 0
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and np.array_equal(a[1], b[1]), name


@pytest.mark.parametrize("seed", list(range(1000, 1008)) + list(range(2000, 2008)))
def test_no_unwritten_hit_fields_fuzz(torch_cuda, checked, seed):
    from tests.test_gpu_fuzz import fuzz_scene

    kind = 4 if seed >= 2000 else None
    sc, cam, rs, tag = fuzz_scene(seed, kind=kind)
    a = gpu_render(torch_cuda, checked, sc, cam, rs)
    assert a[2]["hit_check_failures"] == 0, tag
