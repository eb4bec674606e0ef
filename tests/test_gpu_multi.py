"""Multi-device contexts through the C ABI (octpt_create_multi): one context over a device
list, the tiles dealt round-robin over the entries, gathered with peer copies into the caller's buffers on
the first device.  On the one-GPU box the list repeats device 0 (two or three entries on one GPU, each a
context with its own stream and scene replica), which runs the whole scatter / render / gather path; the
results must be bit-identical to one context's: radiance, per-pixel segment counts and statistics."""
import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

SAME = ("paths", "segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads",
        "block_tests", "beam_restarts")


@pytest.fixture(scope="module")
def multi2(torch_cuda):
    from octree_pathtracing_amd.renderer import HipRenderer

    r = HipRenderer(devices=[0, 0])
    assert r.device_entries == 2
    yield r
    r.close()


@pytest.fixture(scope="module")
def multi3(torch_cuda):
    from octree_pathtracing_amd.renderer import HipRenderer

    r = HipRenderer(devices=[0, 0, 0])
    assert r.device_entries == 3
    yield r
    r.close()


def _same(a, b, tag):
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)), f"{tag}: radiance"
    assert np.array_equal(a[1], b[1]), f"{tag}: segment counts"
    for k in SAME:
        assert a[2][k] == b[2][k], (tag, k, a[2][k], b[2][k])


@pytest.mark.parametrize("name,res", [("tiny", None), ("C3", (480, 270, 4)), ("C4", (256, 144, 2)),
                                      ("C5b", (256, 144, 2)), ("blocks", None), ("C1", None)])
def test_multi_equals_single(torch_cuda, renderer, multi2, multi3, name, res):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    one = gpu_render(torch_cuda, renderer, sc, cam, rs)
    _same(gpu_render(torch_cuda, multi2, sc, cam, rs), one, name + " x2")
    _same(gpu_render(torch_cuda, multi3, sc, cam, rs), one, name + " x3")


def test_multi_shards_progressive_preview(torch_cuda, renderer, multi3):
    """A caller shard (compact tile buffer) split again over the entries; a progressive continuation
    (the running mean and segment counts scattered to the entries and gathered back); preview mode;
    the megakernel; a branch schedule (C20)."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("C3")
    rs.width, rs.height, rs.spp = 203, 117, 2  # ragged tiles
    for k in range(3):
        a = gpu_render(torch_cuda, multi3, sc, cam, rs, shard=(k, 3), compact=True)
        b = gpu_render(torch_cuda, renderer, sc, cam, rs, shard=(k, 3), compact=True)
        _same(a, b, f"shard {k}")
    first = gpu_render(torch_cuda, multi3, sc, cam, rs)
    a = gpu_render(torch_cuda, multi3, sc, cam, rs, spp_start=2, accum=first[0])
    b = gpu_render(torch_cuda, renderer, sc, cam, rs, spp_start=2, accum=first[0])
    _same(a, b, "progressive")
    _same(gpu_render(torch_cuda, multi3, sc, cam, rs, preview=True),
          gpu_render(torch_cuda, renderer, sc, cam, rs, preview=True), "preview")
    _same(gpu_render(torch_cuda, multi3, sc, cam, rs, megakernel=True),
          gpu_render(torch_cuda, renderer, sc, cam, rs, megakernel=True), "megakernel")
    rs.spp = 8
    _same(gpu_render(torch_cuda, multi3, sc, cam, rs, branch_count=4),
          gpu_render(torch_cuda, renderer, sc, cam, rs, branch_count=4), "branch_count 4")


def test_multi_host_and_async_paths(torch_cuda, renderer, multi2):
    """octpt_render (host buffers, tone map) and the RenderingBackend surface (render_frame -> FrameInFlight)
    on a two-entry context equal one context's; the closest-hit query runs on the first entry."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("tiny")
    for r in (renderer, multi2):
        r.set_scene(sc)
        r.set_camera(cam)
    a, ra = multi2.render(rs, with_rgba=True)
    b, rb = renderer.render(rs, with_rgba=True)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32)) and np.array_equal(ra, rb)
    imgs = []
    for r in (multi2, renderer):
        r.set_resolution((rs.width, rs.height))
        r.max_depth, r.seed = rs.max_depth, rs.seed
        r.set_target_spp(3)
        imgs.append((r.render_frame().wait_for(), r.get_float_image().copy()))
    assert np.array_equal(imgs[0][0], imgs[1][0]) and np.array_equal(imgs[0][1].view(np.uint32), imgs[1][1].view(np.uint32))
    rng = np.random.default_rng(5)
    o = rng.uniform(0, 32, (4096, 3)).astype(np.float32)
    d = rng.normal(size=(4096, 3)).astype(np.float32)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    rays = np.concatenate([o, d], 1)
    for x, y in zip(multi2.intersect(rays), renderer.intersect(rays)):
        assert np.array_equal(x, y)


def test_multi_beam_on(torch_cuda):
    """The shipped default (beam on) on a two-entry context: each entry computes its own tiles' beam starts."""
    import os

    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import HipRenderer

    old = os.environ.get("OCTPT_BEAM")
    os.environ["OCTPT_BEAM"] = "1"  # read when a context is created
    try:
        one, two = HipRenderer(device=0), HipRenderer(devices=[0, 0])
    finally:
        if old is None:
            del os.environ["OCTPT_BEAM"]
        else:
            os.environ["OCTPT_BEAM"] = old
    sc, cam, rs = S.make_config("C3")
    rs.width, rs.height, rs.spp = 480, 270, 2
    _same(gpu_render(torch_cuda, two, sc, cam, rs), gpu_render(torch_cuda, one, sc, cam, rs), "beam x2")
    two.close()
    one.close()


def test_multi_poll_cancel_and_errors(torch_cuda, multi3):
    """FrameInFlight on a three-entry context: poll until ready, cancel a long frame (every entry's render
    stops, the accumulation is untouched), and an entry's error reaches the caller with its message."""
    from octree_pathtracing_amd import _lib
    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import FrameInFlightPoll

    sc, cam, rs = S.make_config("tiny")
    multi3.set_scene(sc)
    multi3.set_camera(cam)
    multi3.set_resolution((rs.width, rs.height))
    multi3.max_depth, multi3.seed = rs.max_depth, rs.seed
    multi3.reset_render()
    f = multi3.render_frame(spp_count=rs.spp)
    while True:
        state, payload = f.poll()
        if state is not FrameInFlightPoll.NotReady:
            break
    assert state is FrameInFlightPoll.Ready and multi3.get_current_spp() == rs.spp
    before = multi3.get_float_image().copy()
    f2 = multi3.render_frame(spp_count=512)
    f2.cancel()
    while True:
        state, payload = f2.poll()
        if state is not FrameInFlightPoll.NotReady:
            break
    assert state is FrameInFlightPoll.Cancelled and payload is None
    assert multi3.get_current_spp() == rs.spp
    assert np.array_equal(multi3.get_float_image().view(np.uint32), before.view(np.uint32))
    # a branch schedule that does not end on a pass boundary is refused by every entry (C20)
    multi3.branch_count = 10
    rs.spp = 5  # passes of weight 1, 1, 1, 1, then 6: 5 samples end inside a pass
    with pytest.raises(_lib.OctptError, match="pass boundary"):
        multi3.render(rs)
    multi3.branch_count = 1
