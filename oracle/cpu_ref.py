"""ctypes binding of oracle/libcpu_ref.so -- the CPU restatement of the reference hot path.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() (as the checker) and
bench.py's cpu_baseline leg.  Never imported by the product package.  Parity status: see
oracle/cpu_ref.h ("parity unpinned" for the path tracer; Morton pinned by the reference's tests).
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB_PATH = HERE / "libcpu_ref.so"


def build() -> Path:
    subprocess.run(["make", "-s", "-C", str(HERE)], check=True)
    return LIB_PATH


class RefCamera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("dir", C.c_float * 3), ("up", C.c_float * 3), ("fov", C.c_float)]


class RefMaterial(C.Structure):
    _fields_ = [("ior", C.c_float), ("specular", C.c_float), ("emittance", C.c_float), ("roughness", C.c_float),
                ("metalness", C.c_float), ("texture_index", C.c_uint32), ("tint_index", C.c_uint32),
                ("flags", C.c_uint32)]


class RefTexture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("rgba", C.c_uint8 * 4), ("width", C.c_uint32), ("height", C.c_uint32),
                ("offset", C.c_uint64)]


class RefSun(C.Structure):
    _fields_ = [("azimuth", C.c_float), ("altitude", C.c_float), ("radius", C.c_float), ("color", C.c_float * 4),
                ("apparent_color", C.c_float * 3), ("draw_texture", C.c_int32), ("texture_modification", C.c_int32),
                ("importance_sample_chance", C.c_float), ("importance_sample_radius", C.c_float),
                ("luminosity", C.c_float), ("texture_rgba", C.c_uint8 * 4), ("importance_sampling", C.c_int32),
                ("diffuse_sun", C.c_int32), ("sun_sampling", C.c_int32), ("strict_direct_light", C.c_int32),
                ("sun_luminosity", C.c_int32), ("luminosity_pdf", C.c_float)]


class RefScene(C.Structure):
    _fields_ = [("octant_mask", C.c_void_p), ("octant_children", C.c_void_p), ("n_octants", C.c_uint32),
                ("root", C.c_uint32), ("depth", C.c_uint32), ("leaf_first", C.c_void_p), ("leaf_count", C.c_void_p),
                ("leaf_prims", C.c_void_p), ("n_leaves", C.c_uint32), ("spheres", C.c_void_p),
                ("sphere_material", C.c_void_p), ("n_spheres", C.c_uint32), ("cuboids", C.c_void_p),
                ("cuboid_material", C.c_void_p), ("n_cuboids", C.c_uint32), ("materials", C.c_void_p),
                ("n_materials", C.c_uint32), ("textures", C.c_void_p), ("n_textures", C.c_uint32),
                ("texels", C.c_void_p), ("sun", RefSun), ("emitters_enabled", C.c_int32),
                ("f_sub_surface", C.c_float), ("cuboid_model", C.c_void_p), ("model_quads", C.c_void_p),
                ("n_models", C.c_uint32), ("quads", C.c_void_p), ("n_quads", C.c_uint32),
                ("block_mat", C.c_void_p), ("block_model", C.c_void_p), ("n_blocks", C.c_uint32)]


class RefParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp_start", C.c_uint32), ("spp_count", C.c_uint32),
                ("max_depth", C.c_uint32), ("branch_count", C.c_uint32), ("seed", C.c_uint32),
                ("threads", C.c_uint32), ("forward_accumulation", C.c_int32), ("row_begin", C.c_uint32),
                ("row_end", C.c_uint32), ("preview", C.c_int32)]


class RefStats(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("paths", "segments", "esvo_steps", "node_fetches", "prim_tests",
                                           "leaf_visits", "shade_events", "texel_reads", "max_path_segs",
                                           "block_tests")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class RefOctree(C.Structure):
    _fields_ = [("octant_mask", C.c_void_p), ("octant_children", C.c_void_p), ("n_octants", C.c_uint32),
                ("root", C.c_uint32), ("depth", C.c_uint32), ("leaf_first", C.c_void_p), ("leaf_count", C.c_void_p),
                ("leaf_prims", C.c_void_p), ("n_leaves", C.c_uint32), ("n_leaf_prims", C.c_uint32)]


_lib = None


def load(path: str | Path | None = None) -> C.CDLL:
    """Bind the oracle library (the portable x86-64-v2 build; bench.py's CPU baseline passes its
    -O3 -march=native build of the same source, which then serves every later call)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is None and not LIB_PATH.exists():
        build()
    lib = C.CDLL(str(path or LIB_PATH))
    f, u32, vp = C.c_float, C.c_uint32, C.c_void_p
    for name in ("ref_math_sin", "ref_math_cos", "ref_math_asin", "ref_math_acos"):
        getattr(lib, name).restype = f
        getattr(lib, name).argtypes = [f]
    lib.ref_math_atan2.restype = f
    lib.ref_math_atan2.argtypes = [f, f]
    lib.ref_math_hypot.restype = f
    lib.ref_math_hypot.argtypes = [f, f]
    lib.ref_rng_path_state.restype = u32
    lib.ref_rng_path_state.argtypes = [u32, u32, u32]
    lib.ref_rng_next.restype = f
    lib.ref_rng_next.argtypes = [C.POINTER(u32)]
    lib.ref_morton_encode.restype = C.c_uint64
    lib.ref_morton_encode.argtypes = [C.c_uint64] * 3
    lib.ref_morton_encode_lut.restype = C.c_uint64
    lib.ref_morton_encode_lut.argtypes = [C.c_uint64] * 3
    lib.ref_morton_decode.restype = None
    lib.ref_morton_decode.argtypes = [C.c_uint64] + [C.POINTER(C.c_uint64)] * 3
    lib.ref_morton_lut_selftest.restype = C.c_uint64
    lib.ref_morton_lut_selftest.argtypes = [u32]
    lib.ref_build_octree.restype = C.c_int
    lib.ref_build_octree.argtypes = [vp, u32, vp, u32, u32, u32, C.POINTER(RefOctree)]
    lib.ref_free_octree.restype = None
    lib.ref_free_octree.argtypes = [C.POINTER(RefOctree)]
    lib.ref_intersect.restype = None
    lib.ref_intersect.argtypes = [C.POINTER(RefScene), vp, vp, vp, u32, vp, vp, vp, vp]
    lib.ref_intersect_brute.restype = None
    lib.ref_intersect_brute.argtypes = [C.POINTER(RefScene), vp, u32, vp, vp]
    lib.ref_quad_hit.restype = None
    lib.ref_quad_hit.argtypes = [vp, vp, vp, u32, vp, vp]
    lib.ref_branch_count.restype = u32
    lib.ref_branch_count.argtypes = [u32, u32]
    lib.ref_rng_branch_state.restype = u32
    lib.ref_rng_branch_state.argtypes = [u32, u32]
    lib.ref_render.restype = C.c_int
    lib.ref_render.argtypes = [C.POINTER(RefScene), C.POINTER(RefCamera), C.POINTER(RefParams), vp, vp,
                               C.POINTER(RefStats)]
    lib.ref_tonemap.restype = None
    lib.ref_tonemap.argtypes = [vp, u32, vp]
    lib.ref_lut_float.restype = f
    lib.ref_lut_float.argtypes = [u32]
    lib.ref_lut_byte.restype = C.c_uint8
    lib.ref_lut_byte.argtypes = [u32]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None and a.size else None


def build_octree(spheres: np.ndarray, cuboids: np.ndarray, depth: int, compact: bool = False):
    """Oracle builder -> dict of numpy arrays (octant_mask, octant_children, root, depth, leaf_*).
    compact: merge eight equal sibling leaves bottom-up (Octant::is_compactable, new_octree.rs:227-233)."""
    lib = load()
    sp = np.ascontiguousarray(spheres, np.float32).reshape(-1, 4)
    cb = np.ascontiguousarray(cuboids, np.float32).reshape(-1, 6)
    t = RefOctree()
    rc = lib.ref_build_octree(_p(sp), len(sp), _p(cb), len(cb), depth, 1 if compact else 0, C.byref(t))
    if rc != 0:
        raise RuntimeError(f"ref_build_octree failed ({rc})")
    try:
        def arr(ptr, n, dt, shape=None):
            if n == 0:
                return np.zeros(shape or (0,), dt)
            a = np.frombuffer(C.string_at(ptr, n * np.dtype(dt).itemsize), dtype=dt).copy()
            return a.reshape(shape) if shape else a

        out = dict(octant_mask=arr(t.octant_mask, t.n_octants, np.uint16),
                   octant_children=arr(t.octant_children, 8 * t.n_octants, np.uint32, (t.n_octants, 8)),
                   root=t.root, depth=t.depth,
                   leaf_first=arr(t.leaf_first, t.n_leaves, np.uint32),
                   leaf_count=arr(t.leaf_count, t.n_leaves, np.uint32),
                   leaf_prims=arr(t.leaf_prims, t.n_leaf_prims, np.uint32))
    finally:
        lib.ref_free_octree(C.byref(t))
    return out


class OracleScene:
    """Holds the ctypes RefScene and every array it points to."""

    def __init__(self, scene):
        t = scene.octree
        self._keep = []

        def k(a, dt):
            a = np.ascontiguousarray(a, dt)
            self._keep.append(a)
            return a

        mask = k(t.octant_mask, np.uint16)
        ch = k(t.octant_children, np.uint32)
        lf, lc, lp = k(t.leaf_first, np.uint32), k(t.leaf_count, np.uint32), k(t.leaf_prims, np.uint32)
        sp = k(scene.spheres, np.float32)
        sm = k(scene.sphere_material, np.uint32)
        cb = k(scene.cuboids, np.float32)
        cm = k(scene.cuboid_material, np.uint32)
        mats = (RefMaterial * len(scene.materials))(*[
            RefMaterial(m.ior, m.specular, m.emittance, m.roughness, m.metalness, m.texture_index, m.tint_index,
                        m.flags) for m in scene.materials])
        texs = (RefTexture * len(scene.textures))()
        pool = []
        off = 0
        for i, tx in enumerate(scene.textures):
            texs[i].kind = tx.kind
            texs[i].rgba[:] = list(tx.rgba)
            if tx.kind == 1:
                px = np.ascontiguousarray(tx.pixels, np.uint8)
                texs[i].width, texs[i].height, texs[i].offset = px.shape[1], px.shape[0], off
                pool.append(px.reshape(-1))
                off += px.size
        texels = k(np.concatenate(pool) if pool else np.zeros(1, np.uint8), np.uint8)
        self._keep += [mats, texs]
        s = scene.sun
        st = scene.strategy
        sun = RefSun(s.azimuth, s.altitude, s.radius, (C.c_float * 4)(*s.color), (C.c_float * 3)(*s.apparent_color),
                     int(s.draw_texture), int(s.texture_modification), s.importance_sample_chance,
                     s.importance_sample_radius, s.luminosity, (C.c_uint8 * 4)(*s.texture_rgba),
                     int(st.importance_sampling), int(st.diffuse_sun), int(st.sun_sampling),
                     int(st.strict_direct_light), int(st.sun_luminosity), s.luminosity_pdf)
        self.s = RefScene(_p(mask), _p(ch), len(mask), t.root, t.depth, _p(lf), _p(lc), _p(lp), len(lf), _p(sp), _p(sm),
                          len(sp), _p(cb), _p(cm), len(cb), C.cast(mats, C.c_void_p), len(scene.materials),
                          C.cast(texs, C.c_void_p), len(scene.textures), _p(texels), sun, int(scene.emitters_enabled),
                          scene.f_sub_surface)
        blocks = getattr(scene, "blocks", None)
        if (scene.cuboid_model is not None and len(scene.cuboids)) or blocks is not None:
            if scene.cuboid_model is not None and len(scene.cuboids):
                self.s.cuboid_model = _p(k(scene.cuboid_model, np.uint32))
            mq = k(np.asarray(scene.models, np.uint32).reshape(-1, 2), np.uint32)
            self.s.model_quads = _p(mq)
            self.s.n_models = len(mq)
            qd = np.ascontiguousarray(scene.quads)
            self._keep.append(qd)
            self.s.quads = qd.ctypes.data if len(qd) else None
            self.s.n_quads = len(qd)
        if blocks is not None:  # block-value leaves
            self.s.block_mat = _p(k(np.asarray(blocks, np.uint32).reshape(-1, 6), np.uint32))
            bm = scene.block_model if scene.block_model is not None else np.full(len(blocks), 0xFFFFFFFF, np.uint32)
            self.s.block_model = _p(k(bm, np.uint32))
            self.s.n_blocks = len(blocks)


def render(scene, camera, width, height, spp, *, spp_start=0, max_depth=5, seed=1, threads=8, forward=False,
           accum=None, rows=None, branch_count=1, preview=False):
    """TileRenderer progressive render on the CPU: returns (accum[H,W,4], seg_count[H,W], stats).
    preview=True: RendererMode::Preview (one un-jittered flat-shaded pass, rgb replaced; spp ignored)."""
    lib = load()
    os_ = OracleScene(scene)
    cam = RefCamera((C.c_float * 3)(*camera.eye), (C.c_float * 3)(*camera.direction), (C.c_float * 3)(*camera.up),
                    camera.fov)
    if accum is None:
        accum = np.zeros((height, width, 4), np.float32)
        accum[..., 3] = 1.0
    accum = np.ascontiguousarray(accum, np.float32)
    segs = np.zeros((height, width), np.uint32)
    r0, r1 = rows if rows else (0, height)
    p = RefParams(width, height, spp_start, spp, max_depth, branch_count, seed, threads, int(forward), r0, r1,
                  int(preview))
    st = RefStats()
    rc = lib.ref_render(C.byref(os_.s), C.byref(cam), C.byref(p), _p(accum), _p(segs), C.byref(st))
    if rc != 0:
        raise RuntimeError(f"ref_render failed ({rc})")
    return accum, segs, st.as_dict()


def traversal_data(scene, ray, max_dst=1024.0):
    """Octree::get_traversal_data: (start octant, scale, index_stack[24], time_stack[24])."""
    lib = load()
    os_ = OracleScene(scene)
    r = np.ascontiguousarray(ray, np.float32).reshape(6)
    start, scale = C.c_uint32(), C.c_uint32()
    idx = np.zeros(24, np.uint32)
    ts = np.zeros(24, np.float32)
    lib.ref_traversal_data(C.byref(os_.s), _p(r), C.c_float(max_dst), C.byref(start), C.byref(scale), _p(idx),
                           _p(ts))
    return start.value, scale.value, idx, ts


def intersect(scene, rays, last_prim=None, last_normal=None):
    lib = load()
    os_ = OracleScene(scene)
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = len(rays)
    t = np.zeros(n, np.float32)
    prim = np.zeros(n, np.uint32)
    nrm = np.zeros((n, 3), np.float32)
    steps = np.zeros(n, np.uint32)
    lp = None if last_prim is None else np.ascontiguousarray(last_prim, np.uint32)
    ln = None if last_normal is None else np.ascontiguousarray(last_normal, np.float32)
    lib.ref_intersect(C.byref(os_.s), _p(rays), _p(lp), _p(ln), n, _p(t), _p(prim), _p(nrm), _p(steps))
    return t, prim, nrm, steps


def intersect_brute(scene, rays):
    lib = load()
    os_ = OracleScene(scene)
    rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 6)
    n = len(rays)
    t = np.zeros(n, np.float32)
    prim = np.zeros(n, np.uint32)
    lib.ref_intersect_brute(C.byref(os_.s), _p(rays), n, _p(t), _p(prim))
    return t, prim


def quad_hit(quad_row, rays, voxel):
    """Quad::hit of one octpt_quad row (numpy QUAD_DTYPE record) for rays [n, 6] at `voxel`:
    (t, alpha, beta) [n, 3] and hit flags [n]."""
    lib = load()
    q = np.ascontiguousarray(np.asarray([quad_row]))
    r = np.ascontiguousarray(rays, np.float32)
    v = np.ascontiguousarray(voxel, np.float32)
    n = len(r)
    out = np.zeros((n, 3), np.float32)
    hit = np.zeros(n, np.uint8)
    lib.ref_quad_hit(q.ctypes.data, _p(r), _p(v), n, _p(out), _p(hit))
    return out, hit.astype(bool)


def tonemap(accum):
    lib = load()
    a = np.ascontiguousarray(accum, np.float32)
    n = a.size // 4
    out = np.zeros(a.shape[:-1] + (4,), np.uint8)
    lib.ref_tonemap(_p(a), n, _p(out))
    return out
