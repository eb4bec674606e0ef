"""CPU tests of the oracle (oracle/cpu_ref.c): pinned where the reference pins anything (its own
Morton tests, new_octree.rs:866-884), cross-checked against independent numpy / pure-Python
restatements everywhere else.  Hot-path parity is otherwise unpinned by the reference (SURVEY.md
§8c), see DESIGN.md §2."""
import ctypes as C
import math

import numpy as np
import pytest

from oracle import cpu_ref
from octree_pathtracing_amd import scene as S

F32 = np.float32


@pytest.fixture(scope="module")
def lib():
    return cpu_ref.load()


# ----------------------------------------------------------------------------- Morton (reference KATs)
def _part_by_2(v: int) -> int:  # independent bit loop, not the reference's magic-mask form
    out = 0
    for b in range(21):
        out |= ((v >> b) & 1) << (3 * b)
    return out


def test_morton_code_bit_pattern(lib):
    """new_octree.rs:866-875: encode_morton(1, 0, 1) round-trips through decode_morton."""
    code = lib.ref_morton_encode(1, 0, 1)
    assert code == 0b101  # x -> bit 0, y -> bit 1, z -> bit 2 (new_octree.rs:753-755)
    x, y, z = C.c_uint64(), C.c_uint64(), C.c_uint64()
    lib.ref_morton_decode(code, C.byref(x), C.byref(y), C.byref(z))
    assert (x.value, y.value, z.value) == (1, 0, 1)


def test_morton_encode_matches_bit_loop(lib):
    rng = np.random.default_rng(5)
    for x, y, z in rng.integers(0, 1 << 21, size=(2000, 3)):
        x, y, z = int(x), int(y), int(z)
        want = _part_by_2(x) | (_part_by_2(y) << 1) | (_part_by_2(z) << 2)
        assert lib.ref_morton_encode(x, y, z) == want
        dx, dy, dz = C.c_uint64(), C.c_uint64(), C.c_uint64()
        lib.ref_morton_decode(want, C.byref(dx), C.byref(dy), C.byref(dz))
        assert (dx.value, dy.value, dz.value) == (x, y, z)


def test_morton_code_lut_full_cube(lib):
    """new_octree.rs:876-884: encode_morton == encode_morton_lut on every x, y, z in [0, 1024)^3."""
    assert lib.ref_morton_lut_selftest(1024) == 0


# ----------------------------------------------------------------------------- RNG [C10]
def _lowbias32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _path_state(seed, pixel, sample):
    h = _lowbias32(seed ^ 0xA511E9B3)
    h = _lowbias32(h ^ pixel)
    return _lowbias32(h ^ ((sample * 0x9E3779B9) & 0xFFFFFFFF))


def _next(s):
    s = (s * 747796405 + 2891336453) & 0xFFFFFFFF
    w = (((s >> ((s >> 28) + 4)) ^ s) * 277803737) & 0xFFFFFFFF
    w = (w >> 22) ^ w
    return s, float(np.float32(w >> 8) * np.float32(1.0 / 16777216.0))


def test_rng_matches_python_restatement(lib):
    for seed, pixel, sample in [(1, 0, 0), (1, 2073599, 255), (7, 12345, 3), (0xFFFFFFFF, 1, 1 << 20)]:
        st = lib.ref_rng_path_state(seed, pixel, sample)
        assert st == _path_state(seed, pixel, sample)
        s = C.c_uint32(st)
        ps = st
        for _ in range(16):
            v = lib.ref_rng_next(C.byref(s))
            ps, want = _next(ps)
            assert s.value == ps and v == want and 0.0 <= v < 1.0


def test_rng_uniformity(lib):
    s = C.c_uint32(lib.ref_rng_path_state(3, 99, 0))
    v = np.array([lib.ref_rng_next(C.byref(s)) for _ in range(20000)])
    assert abs(v.mean() - 0.5) < 0.01 and abs(v.var() - 1 / 12) < 0.005


# ----------------------------------------------------------------------------- LUTs (texture.rs:42-62)
def test_luts(lib):
    for i in range(256):
        f = np.float32(np.float32(i) / np.float32(255.0))
        want_f = F32(math.pow(float(f), float(F32(2.2))))
        assert abs(lib.ref_lut_float(i) - want_f) <= 2 * np.spacing(want_f) + 1e-30
        b = F32(math.pow(float(f), float(F32(1.0) / F32(2.2)))) * F32(255.0)
        assert abs(int(lib.ref_lut_byte(i)) - int(min(max(b, 0), 255))) <= 1
    assert lib.ref_lut_byte(0) == 0 and lib.ref_lut_byte(255) == 255


# ----------------------------------------------------------------------------- portable math [C11]
def _ulp_err(got, want):
    want32 = np.float32(want)
    return abs(float(got) - want) / float(np.spacing(np.abs(want32)) or np.float32(1e-45))


@pytest.mark.parametrize("fn,lo,hi,np_fn,bound", [
    ("sin", -7.0, 7.0, math.sin, 4.0), ("cos", -7.0, 7.0, math.cos, 4.0),
    ("asin", -1.0, 1.0, math.asin, 4.0), ("acos", -1.0, 1.0, math.acos, 4.0)])
def test_math_unary_accuracy(lib, fn, lo, hi, np_fn, bound):
    f = getattr(lib, f"ref_math_{fn}")
    xs = np.linspace(lo, hi, 4001, dtype=np.float32)
    worst = 0.0
    for x in xs:
        got = f(float(x))
        want = np_fn(float(x))
        if abs(want) < 1e-6:
            assert abs(got - want) < 1e-6
            continue
        worst = max(worst, _ulp_err(got, want))
    assert worst <= bound, f"{fn}: {worst} ulp"


def test_math_atan2_hypot(lib):
    rng = np.random.default_rng(1)
    pts = rng.uniform(-3, 3, size=(3000, 2)).astype(np.float32)
    worst = 0.0
    for y, x in pts:
        got = lib.ref_math_atan2(float(y), float(x))
        worst = max(worst, _ulp_err(got, math.atan2(float(y), float(x))))
        h = lib.ref_math_hypot(float(x), float(y))
        assert h == float(np.sqrt(np.float32(x) * np.float32(x) + np.float32(y) * np.float32(y)))
    assert worst <= 4.0
    assert lib.ref_math_atan2(0.0, -1.0) == pytest.approx(math.pi, abs=1e-6)


# ----------------------------------------------------------------------------- primitives
def _single_sphere_scene(c, r, depth=6):
    sc = S.Scene()
    ids = S.primitive_materials(sc)
    sc.spheres = np.array([[*c, r]], np.float32)
    sc.sphere_material = np.array([ids["diffuse"][0]], np.uint32)
    sc.build_octree(depth)
    return sc


def test_sphere_kat_numpy(lib):
    """Sphere::hit restated (sphere.rs:33-57, contract C2) in numpy float32, op for op."""
    c, r = (np.float32(32.5), np.float32(30.25), np.float32(31.0)), np.float32(5.5)
    sc = _single_sphere_scene(c, r)
    rng = np.random.default_rng(2)
    o = np.stack([rng.uniform(1, 63, 300), rng.uniform(1, 63, 300), np.full(300, 2.0)], 1).astype(np.float32)
    tgt = np.array(c, np.float32) + rng.uniform(-4, 4, (300, 3)).astype(np.float32)
    d = (tgt - o).astype(np.float32)
    d = d * (np.float32(1) / np.sqrt((d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]))[:, None]
    rays = np.concatenate([o, d], 1).astype(np.float32)
    t, prim, nrm, _ = cpu_ref.intersect(sc, rays)
    cc = np.array(c, np.float32)
    oc = cc[None, :] - o
    a = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    h = (d[:, 0] * oc[:, 0] + d[:, 1] * oc[:, 1]) + d[:, 2] * oc[:, 2]
    q = ((oc[:, 0] * oc[:, 0] + oc[:, 1] * oc[:, 1]) + oc[:, 2] * oc[:, 2]) - r * r
    disc = h * h - a * q
    hit = disc >= 0
    t0 = (h - np.sqrt(np.maximum(disc, 0))) / a
    assert hit.sum() > 200
    assert np.array_equal(prim[hit], np.zeros(hit.sum(), np.uint32))
    assert np.array_equal(t[hit], t0[hit])  # bit-exact
    assert np.all(prim[~hit] == 0xFFFFFFFF)
    p = o[hit] + d[hit] * t0[hit][:, None]
    n_want = (p - cc[None, :]) / r
    assert np.array_equal(nrm[hit], n_want.astype(np.float32))


def test_cuboid_slab_kat(lib):
    """AABB::intersects_new (aabb.rs:172-191, contract C3) on axis-aligned rays: exact face distances."""
    sc = S.Scene()
    ids = S.primitive_materials(sc)
    sc.cuboids = np.array([[10.0, 12.0, 14.0, 20.0, 22.0, 24.0]], np.float32)
    sc.cuboid_material = np.full((1, 6), ids["diffuse"][0], np.uint32)
    sc.build_octree(5)
    rays = np.array([[2, 15, 16, 1, 0, 0], [30, 15, 16, -1, 0, 0], [15, 1, 16, 0, 1, 0],
                     [15, 30, 16, 0, -1, 0], [15, 16, 2, 0, 0, 1], [15, 16, 31, 0, 0, -1]], np.float32)
    t, prim, nrm, _ = cpu_ref.intersect(sc, rays)
    assert np.array_equal(prim, np.full(6, 0x80000000, np.uint32))
    assert np.array_equal(t, np.array([8, 10, 11, 8, 12, 7], np.float32))
    want_n = np.array([[-1, 0, 0], [1, 0, 0], [0, -1, 0], [0, 1, 0], [0, 0, -1], [0, 0, 1]], np.float32)
    assert np.array_equal(nrm, want_n)


# ----------------------------------------------------------------------------- ESVO vs brute force [C1]
@pytest.mark.parametrize("depth,n", [(4, 30), (6, 120), (7, 400)])
def test_esvo_matches_brute_force(depth, n):
    world = float(1 << depth)
    sc = S.Scene()
    ids = S.primitive_materials(sc)
    sc.spheres = S.random_spheres(depth, n, world, 0.3, world / 12)
    sc.sphere_material = np.full(n, ids["diffuse"][0], np.uint32)
    sc.cuboids = S.random_cuboids(depth + 100, n // 10, world, 0.5, world / 10)
    sc.cuboid_material = np.full((n // 10, 6), ids["diffuse"][0], np.uint32)
    sc.build_octree(depth)
    rng = np.random.default_rng(depth)
    m = 1000
    o = rng.uniform(0.01, world - 0.01, (m, 3)).astype(np.float32)
    o[: m // 2] = np.array([world / 2, world / 2, -world / 2], np.float32) + rng.uniform(-1, 1, (m // 2, 3)).astype(np.float32)
    d = rng.normal(size=(m, 3)).astype(np.float32)
    d[: m // 2, 2] = np.abs(d[: m // 2, 2]) + 1.0
    d /= np.linalg.norm(d, axis=1, keepdims=True).astype(np.float32)
    rays = np.concatenate([o, d], 1).astype(np.float32)
    t, prim, _, steps = cpu_ref.intersect(sc, rays)
    tb, pb = cpu_ref.intersect_brute(sc, rays)
    # The octree covers [0, 2^depth)^3 only: a primitive part outside it is invisible to ESVO.
    # Everywhere else ESVO (first accepted hit in leaf order) must equal the global closest root.
    p = o + d * np.where(np.isfinite(tb), tb, 0)[:, None]
    visible = ~np.isfinite(tb) | np.all((p >= 0) & (p < world), axis=1)
    assert visible.mean() > 0.9
    assert np.array_equal(prim[visible], pb[visible])
    assert np.array_equal(t[visible], tb[visible])
    # the closest root lies outside the cube: ESVO reports a miss or a farther visible hit
    far = ~visible & (prim != 0xFFFFFFFF)
    assert np.all(t[far] >= tb[far])
    assert steps.max() < 1000 and steps.min() >= 0


# ----------------------------------------------------------------------------- accumulation order
def test_forward_matches_recursive_accumulation():
    sc, cam, rs = S.make_config("tiny")
    a_rec, seg_rec, st_rec = cpu_ref.render(sc, cam, 48, 32, 2, forward=False, threads=4)
    a_fwd, seg_fwd, st_fwd = cpu_ref.render(sc, cam, 48, 32, 2, forward=True, threads=4)
    assert np.array_equal(seg_rec, seg_fwd)
    assert st_rec["segments"] == st_fwd["segments"] and st_rec["esvo_steps"] == st_fwd["esvo_steps"]
    rel = np.abs(a_rec[..., :3] - a_fwd[..., :3]) / np.maximum(np.abs(a_rec[..., :3]), 1e-3)
    assert rel.max() < 1e-5


def test_progressive_split_identical():
    """Rendering 1+3 passes progressively equals 4 passes at once (running mean order, a1)."""
    sc, cam, rs = S.make_config("tiny")
    full, _, _ = cpu_ref.render(sc, cam, 32, 24, 4, forward=True, threads=4)
    part, _, _ = cpu_ref.render(sc, cam, 32, 24, 1, forward=True, threads=4)
    part, _, _ = cpu_ref.render(sc, cam, 32, 24, 3, spp_start=1, forward=True, threads=4, accum=part)
    assert np.array_equal(full, part)


def test_tonemap_kat(lib):
    acc = np.array([[0, 0, 0, 1], [1, 1, 1, 1], [2, 0.5, 0.25, 0.5]], np.float32)
    out = cpu_ref.tonemap(acc)
    assert out[0].tolist() == [0, 0, 0, 255]
    assert out[1].tolist() == [255, 255, 255, 255]
    assert out[2, 0] == 255 and out[2, 3] == 127
    assert out[2, 1] == lib.ref_lut_byte(int(np.float32(0.5) * np.float32(255)))


def test_preview_restatement():
    """RendererMode::Preview re-derived in numpy from the oracle's own pieces:
    a pixel whose ray misses on its first segment holds get_sky_color_inner + add_sun_color (the
    path-traced depth-0 miss colour of an un-jittered ray), a hit pixel holds
    texel * emittance * max(AMBIENT, n . sw); alpha is left untouched and nothing is random."""
    sc, cam, rs = S.make_config("tiny")
    W, H = 48, 32
    pre = np.zeros((H, W, 4), np.float32)
    pre[..., 3] = 0.25
    acc, seg, st = cpu_ref.render(sc, cam, W, H, 1, threads=2, preview=True, accum=pre.copy())
    acc2, seg2, _ = cpu_ref.render(sc, cam, W, H, 7, seed=99, threads=2, preview=True, accum=pre.copy())
    assert np.array_equal(acc, acc2) and np.array_equal(seg, seg2)  # spp / seed do not apply
    assert np.all(acc[..., 3] == 0.25) and st["shade_events"] == 0 and st["paths"] == W * H
    # the same rays through the closest-hit query: first-segment misses are sky pixels
    dim = float(max(W, H))
    ys, xs = np.mgrid[0:H, 0:W]
    xn = ((2 * xs + 1).astype(np.float32) - np.float32(W)) / np.float32(dim)
    yn = ((2 * (H - ys) - 1).astype(np.float32) - np.float32(H)) / np.float32(dim)
    d_f = np.float32(1.0 / math.tan(cam.fov / 2.0))
    cdir, cup = np.float32(cam.direction), np.float32(cam.up)
    right = np.cross(cdir, cup).astype(np.float32)
    nd = (cdir * d_f)[None, None] + right[None, None] * xn[..., None] + cup[None, None] * yn[..., None]
    dirs = (nd / np.linalg.norm(nd, axis=-1, keepdims=True)).astype(np.float32)
    rays = np.concatenate([np.broadcast_to(np.float32(cam.eye), dirs.shape), dirs], -1).reshape(-1, 6)
    _, prim, nrm, _ = cpu_ref.intersect(sc, rays)
    miss = (prim == 0xFFFFFFFF).reshape(H, W)
    assert miss.any() and (~miss).any()
    assert np.all(seg[miss] == 1)
    sky = acc[miss][:, :3]
    assert np.all((sky == np.float32([0.5, 0.7, 1.0])).all(-1) | (sky > 1.0).all(-1))
    # opaque first hits: flat shading with the sun constants of scene/mod.rs:294-307, 352-353
    az, alt = np.float32(math.pi / 2.5), np.float32(math.pi / 3.0)
    sw = np.float32([math.cos(az) * abs(math.cos(alt)), math.sin(alt), math.sin(az) * abs(math.cos(alt))])
    hit1 = (~miss) & (seg == 1)
    shading = np.maximum(np.float32(0.3), (nrm.reshape(H, W, 3)[hit1] * sw).sum(-1))
    emit = np.float32(1.25) ** np.float32(2.2)
    ratio = acc[hit1][:, :3] / (emit * shading)[:, None]
    assert np.all(ratio >= 0) and np.all(ratio <= 1.0 + 1e-5)  # texel colours in [0, 1]
