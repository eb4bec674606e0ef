"""The lean 24-B path state: a continuing path's radiance is exactly 0 when the scene
has no emitters and no sun sampling, and its chunk item equals its slot when the pool holds the chunk, so
neither is stored (WaveBuffers::lean).  Renders with it equal renders with the 40-B state (OCTPT_LEAN=0) bit
for bit, statistics included, on every scene kind -- the lean state on spheres, boxes, block models, block
values, the beam's retraced camera rays and the drain; the full state where it must stay (emitters, sun
sampling, a pool smaller than the chunk)."""
import os

import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

SAME = ("paths", "segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads",
        "block_tests", "beam_restarts")


def _with_env(env, **kw):
    from octree_pathtracing_amd.renderer import HipRenderer

    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)  # read when the context is created
    try:
        return HipRenderer(**kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def full_state(torch_cuda):
    r = _with_env({"OCTPT_LEAN": "0"}, device=0)
    yield r
    r.close()


@pytest.fixture(scope="module")
def beam_pair(torch_cuda):
    a = _with_env({"OCTPT_BEAM": "1"}, device=0)
    b = _with_env({"OCTPT_BEAM": "1", "OCTPT_LEAN": "0"}, device=0)
    yield a, b
    a.close()
    b.close()


def _same(a, b, tag):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), f"{tag}: radiance"
    assert np.array_equal(a[1], b[1]), f"{tag}: segment counts"
    for k in SAME:
        assert a[2][k] == b[2][k], (tag, k)


@pytest.mark.parametrize("name,res,variant", [
    ("tiny", None, None), ("C3", (480, 270, 4), None), ("C4", (256, 144, 2), None), ("C5", (256, 144, 2), None),
    ("C5b", (256, 144, 2), None), ("blocks-b", None, None), ("C2", (160, 90, 4), "fast"), ("tiny", None, "emit")])
def test_lean_equals_full(torch_cuda, renderer, full_state, name, res, variant):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    if variant == "emit":  # an emitting material: the 40-B state stays
        sc.materials[1].emittance = 5.0
        sc.emitters_enabled = True
    elif variant:
        S.with_sun_variant(sc, variant)
    _same(gpu_render(torch_cuda, renderer, sc, cam, rs), gpu_render(torch_cuda, full_state, sc, cam, rs), name)


def test_lean_with_beam_retrace(torch_cuda, beam_pair):
    """The step-cap world with the beam on: the chunk's first shade stores a retraced camera ray's lean state."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("cap")
    a = gpu_render(torch_cuda, beam_pair[0], sc, cam, rs)
    b = gpu_render(torch_cuda, beam_pair[1], sc, cam, rs)
    _same(a, b, "cap")
    assert a[2]["beam_restarts"] > 0
