"""The tile deal (octpt_set_tile_order / octpt_balance_tiles): a shard owns the 8x8 tiles at
dealing positions k + u * N, and a tile order puts any frame tile at any position.  Per-pixel RNG streams make
the image independent of the deal, so every render under an order must equal the round-robin render bit for
bit -- whole frames, compact shards gathered by the unshard kernel, the camera rays' beam starts, preview,
and a multi-device context -- while the balanced order moves segments between shards."""
import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu

SAME = ("paths", "segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads",
        "block_tests", "beam_restarts")


def _fresh(devices=None, beam=False):
    import os

    from octree_pathtracing_amd.renderer import HipRenderer

    old = os.environ.get("OCTPT_BEAM")
    os.environ["OCTPT_BEAM"] = "1" if beam else "0"
    try:
        return HipRenderer(devices=devices) if devices else HipRenderer(device=0)
    finally:
        if old is None:
            del os.environ["OCTPT_BEAM"]
        else:
            os.environ["OCTPT_BEAM"] = old


def _shuffled(W, H, seed):
    T = ((W + 7) // 8) * ((H + 7) // 8)
    return np.random.default_rng(seed).permutation(T).astype(np.uint32)


def _gather(torch, r, sc, cam, rs, N):
    """Every compact shard rendered in turn, gathered by octpt_unshard_device: (frame, segments per shard)."""
    from octree_pathtracing_amd.renderer import shard_pixels

    W, H = rs.width, rs.height
    stride = max(shard_pixels(W, H, i, N) for i in range(N))
    buf = torch.zeros((N * stride, 4), dtype=torch.float32, device="cuda")
    segs = []
    for i in range(N):
        a, s, st = gpu_render(torch, r, sc, cam, rs, shard=(i, N), compact=True)
        buf[i * stride:i * stride + len(a)] = torch.as_tensor(a, device="cuda")
        segs.append(st["segments"])
    frame = torch.zeros((H * W, 4), dtype=torch.float32, device="cuda")
    r.unshard_device(W, H, N, buf.data_ptr(), stride, frame.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return frame.cpu().numpy().reshape(H, W, 4), segs


@pytest.mark.parametrize("name,res,beam", [("tiny", (70, 45, 4), False), ("C3", (480, 270, 4), True),
                                           ("C5b", (256, 144, 2), True), ("blocks", None, False)])
def test_order_equals_round_robin(torch_cuda, renderer, name, res, beam):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config(name)
    if res:
        rs.width, rs.height, rs.spp = res
    W, H = rs.width, rs.height
    r = _fresh(beam=beam)
    try:
        ref = gpu_render(torch_cuda, r, sc, cam, rs)
        r.set_tile_order(W, H, _shuffled(W, H, 5))
        got = gpu_render(torch_cuda, r, sc, cam, rs)  # whole frame, image layout
        assert np.array_equal(got[0].view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(got[1], ref[1])
        for k in SAME:
            assert got[2][k] == ref[2][k], (name, k)
        for N in (3, 8):
            frame, segs = _gather(torch_cuda, r, sc, cam, rs, N)
            assert np.array_equal(frame.view(np.uint32), ref[0].view(np.uint32)), (name, N)
            assert sum(segs) == ref[2]["segments"]
        prev = gpu_render(torch_cuda, r, sc, cam, rs, preview=True)
        r.set_tile_order(W, H, None)
        prev_ref = gpu_render(torch_cuda, r, sc, cam, rs, preview=True)
        assert np.array_equal(prev[0].view(np.uint32), prev_ref[0].view(np.uint32))
    finally:
        r.close()


def test_balanced_order_moves_segments(torch_cuda, renderer):
    """The order octpt_balance_tiles derives from a render's per-pixel segment counts: the frame is unchanged and
    the most loaded of 8 shards carries fewer segments than under round robin (C3 crop, same samples)."""
    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import balance_tiles

    sc, cam, rs = S.make_config("C3")
    rs.width, rs.height, rs.spp = 480, 272, 4
    W, H = rs.width, rs.height
    r = _fresh(beam=True)
    try:
        full = gpu_render(torch_cuda, r, sc, cam, rs)
        _, rr = _gather(torch_cuda, r, sc, cam, rs, 8)
        r.set_tile_order(W, H, balance_tiles(W, H, 8, full[1]))
        frame, bal = _gather(torch_cuda, r, sc, cam, rs, 8)
        assert np.array_equal(frame.view(np.uint32), full[0].view(np.uint32))
        assert sum(bal) == sum(rr) == full[2]["segments"]
        assert max(bal) < max(rr), (bal, rr)
    finally:
        r.close()


def test_order_multi_device(torch_cuda, renderer):
    """A two-entry context (device 0 twice) under a tile order: whole frame and a caller shard split again over
    the entries, equal to one context's renders."""
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("C3")
    rs.width, rs.height, rs.spp = 200, 120, 2
    W, H = rs.width, rs.height
    order = _shuffled(W, H, 9)
    one = _fresh()
    two = _fresh(devices=[0, 0])
    try:
        one.set_tile_order(W, H, order)
        two.set_tile_order(W, H, order)
        a = gpu_render(torch_cuda, one, sc, cam, rs)
        b = gpu_render(torch_cuda, two, sc, cam, rs)
        assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32)) and np.array_equal(a[1], b[1])
        fa, _ = _gather(torch_cuda, one, sc, cam, rs, 3)
        fb, _ = _gather(torch_cuda, two, sc, cam, rs, 3)
        assert np.array_equal(fa.view(np.uint32), fb.view(np.uint32))
        assert np.array_equal(fa.view(np.uint32), a[0].view(np.uint32))
    finally:
        one.close()
        two.close()


def test_order_validation(torch_cuda, renderer):
    from octree_pathtracing_amd import _lib
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("tiny")
    r = _fresh()
    try:
        T = ((rs.width + 7) // 8) * ((rs.height + 7) // 8)
        with pytest.raises(_lib.OctptError) as e:
            r.set_tile_order(rs.width, rs.height, np.zeros(T, np.uint32))  # not a permutation
        assert e.value.status == _lib.ERR_INVALID_ARG
        r.set_tile_order(rs.width, rs.height, _shuffled(rs.width, rs.height, 1))
        rs2 = S.make_config("tiny")[2]
        rs2.width += 8
        with pytest.raises(_lib.OctptError) as e:  # another frame size while the order is set
            gpu_render(torch_cuda, r, sc, cam, rs2)
        assert e.value.status == _lib.ERR_INVALID_ARG
        r.set_tile_order(rs.width, rs.height, None)
        gpu_render(torch_cuda, r, sc, cam, rs2)
    finally:
        r.close()


def test_order_regeneration_branches_async(torch_cuda, renderer):
    """A tile order under the other paths that map items to pixels: a pool smaller than the chunk (shade
    regenerates camera rays, beam on), a branch schedule (C20), and the asynchronous frame (octpt_render_async)."""
    import os

    from octree_pathtracing_amd import scene as S
    from octree_pathtracing_amd.renderer import HipRenderer

    sc, cam, rs = S.make_config("tiny")
    rs.width, rs.height, rs.spp = 70, 45, 8
    W, H = rs.width, rs.height
    order = _shuffled(W, H, 21)
    old = {k: os.environ.get(k) for k in ("OCTPT_BEAM", "OCTPT_POOL", "OCTPT_CHUNK")}
    os.environ.update(OCTPT_BEAM="1", OCTPT_POOL="4096", OCTPT_CHUNK="8192")
    try:
        small = HipRenderer(device=0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    try:
        for bc in (1, 4):
            ref = gpu_render(torch_cuda, small, sc, cam, rs, branch_count=bc)
            small.set_tile_order(W, H, order)
            got = gpu_render(torch_cuda, small, sc, cam, rs, branch_count=bc)
            small.set_tile_order(W, H, None)
            assert np.array_equal(got[0].view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(got[1], ref[1]), bc
            for k in SAME:
                assert got[2][k] == ref[2][k], (bc, k)
        small.set_scene(sc)
        small.set_camera(cam)
        small.set_resolution((W, H))
        small.max_depth, small.seed = rs.max_depth, rs.seed
        small.branch_count = 1
        want = small.render_frame(spp_count=4).wait_for().copy()
        want_f = np.array(small.get_float_image(), copy=True)
        small.reset_render()
        small.set_tile_order(W, H, order)
        got = small.render_frame(spp_count=4).wait_for()
        assert np.array_equal(got, want)
        assert np.array_equal(np.asarray(small.get_float_image()).view(np.uint32), want_f.view(np.uint32))
    finally:
        small.close()
