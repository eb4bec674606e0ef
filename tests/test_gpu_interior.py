"""Interior cameras (the camera inside the octree: C1, C3-in, C5-fp) against the oracle, render and
preview.  These configs were added for the start-chain experiment (get_traversal_data's beam start,
octree_traversal.rs:537-714 / gpu_renderer.rs:579-581; measured -1 % on C3 / C5 and removed from the
product kernel in round 3, its patch kept as tools/rejected/node_cache_start_chain.patch);
they stay as parity cases for rays that start inside the octree cube."""
import numpy as np
import pytest

from tests.test_gpu_parity import assert_parity, gpu_render, oracle, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,res", [("C1", None), ("C3-in", (192, 108, 2)), ("C5-fp", (192, 108, 1))])
def test_interior_camera_parity(torch_cuda, renderer, name, res):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    assert_parity(gpu_render(torch_cuda, renderer, sc, cam, rs), oracle(sc, cam, rs, forward=True), name)


@pytest.mark.parametrize("name,res", [("C3-in", (256, 144)), ("C5-fp", (320, 180))])
def test_interior_camera_preview_parity(torch_cuda, renderer, name, res):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    rs.width, rs.height = res
    acc, segs, st = gpu_render(torch_cuda, renderer, sc, cam, rs, preview=True)
    racc, rsegs, rst = oracle(sc, cam, rs, preview=True)
    assert np.array_equal(segs, rsegs)
    assert st["segments"] == rst["segments"] and st["esvo_steps"] == rst["esvo_steps"]
    assert np.array_equal(acc, racc)
