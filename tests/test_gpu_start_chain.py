"""Start chain: the descends the camera's centre ray makes from the root
(get_traversal_data's beam start, octree_traversal.rs:537-714 / gpu_renderer.rs:579-581) are replayed
for every ray whose first iterations descend into the same children, with the slots taken from the
chain.  The replay is an exact replica of esvo_step's descend, so renders and previews stay bit-exact
against the oracle (segment counts, ESVO iteration totals, radiance) with the camera inside the octree,
where the chain is long, and equal to renders with the replay switched off (OCTPT_START_CHAIN=0).

The replay measured -1 % on C3 / C5 and +-0 on preview, so the default build compiles it
out (OCTPT_START_CHAIN 0 in octpt_internal.h); these tests then pin the interior-camera configs, and
with a -DOCTPT_START_CHAIN=1 build (scripts/build_variant.py, OCTPT_LIB) they check the replay itself
(profiles/r02/start_chain_*.log: the whole GPU suite green with the replay on)."""
import os
import time

import numpy as np
import pytest

from tests.test_gpu_parity import assert_parity, gpu_render, oracle, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def renderer_off(torch_cuda):
    from octree_pathtracing_amd.renderer import HipRenderer

    old = os.environ.get("OCTPT_START_CHAIN")
    os.environ["OCTPT_START_CHAIN"] = "0"  # read when the context is created
    try:
        r = HipRenderer(device=0)
    finally:
        if old is None:
            del os.environ["OCTPT_START_CHAIN"]
        else:
            os.environ["OCTPT_START_CHAIN"] = old
    yield r
    r.close()


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


@pytest.mark.parametrize("name,res,preview", [("C3", (480, 270, 4), False), ("C3-in", (480, 270, 4), False),
                                              ("C5-fp", (480, 270, 2), False), ("C4", (320, 180, 2), False),
                                              ("C3-in", (1920, 1080, 1), True), ("C5-fp", (3840, 2160, 1), True),
                                              ("blocks", None, False)])
def test_start_chain_off_identical(torch_cuda, renderer, renderer_off, name, res, preview):
    """Replay on == replay off, bit for bit, with both timed (printed) at a moderate size."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    out, ms = [], []
    for r in (renderer, renderer_off):
        gpu_render(torch_cuda, r, sc, cam, rs, preview=preview)  # warm
        t0 = time.perf_counter()
        out.append(gpu_render(torch_cuda, r, sc, cam, rs, preview=preview))
        ms.append((time.perf_counter() - t0) * 1e3)
    (a, sa, sta), (b, sb, stb) = out
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(sa, sb)
    for k in ("segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events"):
        assert sta[k] == stb[k], k
    print(f"\n{name} {'preview' if preview else 'render'} {rs.width}x{rs.height}x{rs.spp}: start chain "
          f"{ms[0]:.2f} ms, off {ms[1]:.2f} ms")
