"""The drain: once every chunk item is claimed and few rays are queued, one launch
finishes the queued paths in-lane instead of one extend / shade pair per remaining segment.  It runs
the wavefront's own per-segment code and record formats, so a render with the drain is bit-identical
to one without it (OCTPT_DRAIN_RAYS=0): radiance, per-pixel segment counts and every statistic, on
sphere, box, sun-sampling and branch-count scenes, and with a pool small enough that several chunks
each end in a drain.  Block-model scenes (C5, blocks) keep the tail iterations; their cases check
that the switch leaves them alone.  Block-value scenes (C23: C5b, blocks-b, C5s-small) drain."""
import os

import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

STATS = ("paths", "segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads",
         "block_tests")


def _renderer_with(env):
    from octree_pathtracing_amd.renderer import HipRenderer

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)  # read when the context is created
    try:
        return HipRenderer(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def no_drain(torch_cuda):
    r = _renderer_with({"OCTPT_DRAIN_RAYS": "0"})
    yield r
    r.close()


@pytest.fixture(scope="module")
def small_pool_drain(torch_cuda):
    r = _renderer_with({"OCTPT_POOL": "65536", "OCTPT_CHUNK": "200000"})
    yield r
    r.close()


def _same(a, b):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), "radiance"
    assert np.array_equal(a[1], b[1]), "segment counts"
    for k in STATS:
        assert a[2][k] == b[2][k], k


@pytest.mark.parametrize("name,res,variant,bc", [("C3", (480, 270, 4), None, 1), ("C2", (320, 180, 8), None, 1),
                                                 ("C4", (256, 144, 2), None, 1), ("C5", (256, 144, 2), None, 1),
                                                 ("blocks", None, None, 1), ("tiny", None, "hq", 1),
                                                 ("C2", (160, 90, 4), "nee_importance", 1), ("tiny", None, None, 4),
                                                 ("C5b", (256, 144, 2), None, 1), ("blocks-b", None, None, 1),
                                                 ("C5s-small", (256, 144, 4), "fast", 1)])
def test_drain_equals_wavefront(torch_cuda, renderer, no_drain, small_pool_drain, name, res, variant, bc):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    if variant:
        S.with_sun_variant(sc, variant)
    if bc > 1:
        rs.spp = 8
    a = gpu_render(torch_cuda, renderer, sc, cam, rs, branch_count=bc)
    b = gpu_render(torch_cuda, no_drain, sc, cam, rs, branch_count=bc)
    _same(a, b)
    c = gpu_render(torch_cuda, small_pool_drain, sc, cam, rs, branch_count=bc)
    _same(a, c)


@pytest.fixture(scope="module")
def drain_models(torch_cuda):
    r = _renderer_with({"OCTPT_DRAIN_MODELS": "1", "OCTPT_POOL": "65536", "OCTPT_CHUNK": "200000"})
    yield r
    r.close()


@pytest.mark.parametrize("name,res", [("C5", (256, 144, 2)), ("blocks", None)])
def test_drain_in_block_model_scenes(torch_cuda, renderer, drain_models, name, res):
    """OCTPT_DRAIN_MODELS=1 (the A/B knob): block-model scenes drained too, with several
    chunks, render bit-identically; the drain ran (its share is in the statistics' drain row)."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    a = gpu_render(torch_cuda, renderer, sc, cam, rs)
    b = gpu_render(torch_cuda, drain_models, sc, cam, rs)
    _same(a, b)
    assert b[2]["drain"]["segments"] > 0
