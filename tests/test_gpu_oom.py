"""Out-of-memory fallback of the wavefront state (octpt_api.cpp ensure_wave /
enqueue_wavefront).  OCTPT_DEVICE_MEM_LIMIT (MiB, read at octpt_create) caps the context's wavefront
allocations so that the fallback runs on an idle GPU:

- queues + path state that do not fit halve the pool (down to 2^20 slots) and the pool obtained
  becomes the context's cap;
- colour records that do not fit halve the chunk;
- the render equals the uncapped one bit for bit (pools and chunks of any size render the same frame),
  and a second render neither re-allocates nor warns again.

The tiny scene at 256x256x32 spp is one 2^21-item chunk: 248 MiB of queues + path state (124 B per
slot: round 5 keeps the lean path state per queue position) and 32 MiB of colour records uncapped."""
import numpy as np
import pytest

from tests.test_gpu_parity import gpu_render, renderer, torch_cuda  # noqa: F401

pytestmark = pytest.mark.gpu


def _scene(variant=None):
    from octree_pathtracing_amd import scene as S

    sc, cam, rs = S.make_config("tiny")
    if variant:
        S.with_sun_variant(sc, variant)
    rs.width, rs.height, rs.spp = 256, 256, 32
    return sc, cam, rs


def _capped(monkeypatch, mib):
    from octree_pathtracing_amd.renderer import HipRenderer

    monkeypatch.setenv("OCTPT_DEVICE_MEM_LIMIT", str(mib))
    r = HipRenderer(device=0)
    monkeypatch.delenv("OCTPT_DEVICE_MEM_LIMIT")
    return r


@pytest.mark.parametrize("mib,variant,pool,chunk", [
    (200, None, 1 << 20, 1 << 21),      # the pool halves, the chunk stays
    (150, None, 1 << 20, 1 << 20),      # then the colour records do not fit either: the chunk halves
    (210, "fast", 1 << 20, 1 << 20),    # sun sampling: + 64 MiB of planes at 2^20 slots, then the chunk
])
def test_oom_fallback_is_stable_and_exact(torch_cuda, renderer, monkeypatch, capfd, mib, variant, pool, chunk):
    sc, cam, rs = _scene(variant)
    ref, rsegs, rst = gpu_render(torch_cuda, renderer, sc, cam, rs)
    capfd.readouterr()
    r = _capped(monkeypatch, mib)
    try:
        a, segs, st = gpu_render(torch_cuda, r, sc, cam, rs)
        err = capfd.readouterr().err
        assert "did not fit" in err
        assert st["pool_slots"] == pool and st["chunk_items"] == chunk, st
        allocs = st["wave_allocs"]
        assert np.array_equal(a.view(np.uint32), ref.view(np.uint32)) and np.array_equal(segs, rsegs)
        for k in ("segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events"):
            assert st[k] == rst[k], k
        # a second render: the same sizes, no re-allocation, no second warning
        b, _, st2 = gpu_render(torch_cuda, r, sc, cam, rs)
        assert capfd.readouterr().err == ""
        assert st2["wave_allocs"] == allocs and st2["pool_slots"] == pool and st2["chunk_items"] == chunk
        assert np.array_equal(b.view(np.uint32), ref.view(np.uint32))
    finally:
        r.close()


def test_oom_floor_fails_cleanly(torch_cuda, monkeypatch):
    """Below the floor (2^20 slots do not fit) the render fails with OOM and a message, no crash."""
    from octree_pathtracing_amd import _lib

    sc, cam, rs = _scene()
    r = _capped(monkeypatch, 64)
    try:
        with pytest.raises(_lib.OctptError) as ei:
            gpu_render(torch_cuda, r, sc, cam, rs)
        assert ei.value.status == _lib.ERR_OOM
        assert r._lib.octpt_last_error(r._ctx)
    finally:
        r.close()
