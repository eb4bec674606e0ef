"""The C ABI driven from a plain C host (tools/capi_host.c, built by __graft_entry__.build()): no Python in the
render path, as the Rust shim of INTEGRATION.md §3 would drive it.  The C program builds a sphere scene with the
library's host builder, uploads it, renders a progressive frame synchronously then asynchronously, and runs a
closest-hit batch; the same scene through the Python bindings must give the same frame and hits bit for bit, and
the oracle the same per-frame statistics and radiance within the parity tolerance."""
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
