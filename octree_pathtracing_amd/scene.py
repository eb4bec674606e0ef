"""Scene model mirroring the reference's Scene / Octree / Material / Texture / Sun / Camera
(reference src/scene/mod.rs:146-156, src/octree/new_octree.rs:13-74,
src/textures/material.rs:185-195, src/textures/texture.rs:15-18, src/scene/mod.rs:271-383,
src/renderer/camera.rs:8-66), plus the seeded synthetic scene generator of BASELINE.json's
configs C1-C5.  All arrays are numpy; the octree is built by the product's
C++ builder (``liboctpt.so: octpt_build_octree``).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from . import _lib

F32 = np.float32
PI = F32(np.pi)  # std::f32::consts::PI

# MaterialFlags (material.rs:99-108)
OPAQUE, SUBSURFACE_SCATTER, REFRACTIVE, WATERLOGGED, SOLID = 0x1, 0x2, 0x4, 0x8, 0x10
DEFAULT_IOR = F32(1.000293)


@dataclass
class Material:
    """GPUMaterial field set (gpu_material.rs:67-76); defaults = MaterialBuilder::build."""
    ior: float = float(DEFAULT_IOR)
    specular: float = 0.0
    emittance: float = 0.0
    roughness: float = 0.0
    metalness: float = 0.0
    texture_index: int = 0
    tint_index: int = 0
    flags: int = OPAQUE | SOLID


def air_material(texture_index: int = 0) -> Material:
    """Material::AIR (material.rs:198-207)."""
    return Material(ior=float(DEFAULT_IOR), flags=0, texture_index=texture_index)


@dataclass
class Texture:
    """Texture::Color(U8Color) or Texture::Image(RTWImage as RGBA8)."""
    kind: int = _lib.TEXTURE_COLOR
    rgba: tuple = (255, 0, 255, 255)  # Texture::DEFAULT_TEXTURE (texture.rs:49)
    pixels: np.ndarray | None = None  # (h, w, 4) uint8 for images

    @staticmethod
    def color(r: int, g: int, b: int, a: int = 255) -> "Texture":
        return Texture(_lib.TEXTURE_COLOR, (r, g, b, a), None)

    @staticmethod
    def image(rgba: np.ndarray) -> "Texture":
        rgba = np.ascontiguousarray(rgba, dtype=np.uint8)
        assert rgba.ndim == 3 and rgba.shape[2] == 4
        return Texture(_lib.TEXTURE_IMAGE, (0, 0, 0, 0), rgba)


@dataclass
class SunSamplingStrategy:
    """SunSamplingStrategy presets (scene/mod.rs:77-127)."""
    sun_sampling: bool = False
    diffuse_sun: bool = True
    strict_direct_light: bool = False
    sun_luminosity: bool = True
    importance_sampling: bool = True


STRATEGY_OFF = SunSamplingStrategy(False, True, False, True, False)
STRATEGY_NON_LUMINOUS = SunSamplingStrategy(False, False, False, False, False)
STRATEGY_FAST = SunSamplingStrategy(True, False, False, False, False)
STRATEGY_IMPORTANCE = SunSamplingStrategy(False, True, False, True, True)
STRATEGY_HIGH_QUALITY = SunSamplingStrategy(True, True, True, True, False)
STRATEGIES = {"OFF": STRATEGY_OFF, "NON_LUMINOUS": STRATEGY_NON_LUMINOUS, "FAST": STRATEGY_FAST,
              "IMPORTANCE": STRATEGY_IMPORTANCE, "HIGH_QUALITY": STRATEGY_HIGH_QUALITY}

# sun-sampling test variants: name -> (strategy, set SUBSURFACE_SCATTER on opaque materials)
SUN_VARIANTS = {
    "fast": (STRATEGY_FAST, False),
    "hq": (STRATEGY_HIGH_QUALITY, False),
    "hq_sss": (STRATEGY_HIGH_QUALITY, True),
    # sun sampling with importance-sampled bounces: the one combination whose weights are kept
    "nee_importance": (SunSamplingStrategy(True, True, False, True, True), False),
}


def with_sun_variant(scene: "Scene", variant: str) -> "Scene":
    """Switch a scene to one of SUN_VARIANTS in place (the octree is unaffected) and return it."""
    strategy, sss = SUN_VARIANTS[variant]
    scene.strategy = SunSamplingStrategy(**vars(strategy))
    if sss:
        for m in scene.materials:
            if m.flags & OPAQUE:
                m.flags |= SUBSURFACE_SCATTER
    return scene


@dataclass
class Sun:
    """Sun::default (scene/mod.rs:294-307) arguments + tunables."""
    azimuth: float = float(PI / F32(2.5))
    altitude: float = float(PI / F32(3.0))
    radius: float = 0.03
    color: tuple = (1.0, 1.0, 1.0, 1.0)
    texture_rgba: tuple = (255, 255, 255, 255)
    draw_texture: bool = True
    texture_modification: bool = False
    apparent_color: tuple = (1.0, 1.0, 1.0)
    importance_sample_chance: float = 0.1
    importance_sample_radius: float = 1.2
    luminosity: float = 100.0
    luminosity_pdf: float = 1.0 / 100.0  # Sun::new hard-codes 1/100 (scene/mod.rs:376)


@dataclass
class Camera:
    """renderer::camera::Camera (camera.rs:8-39); default eye (0,0,10), dir +Z, up +Y, fov 70 deg."""
    eye: tuple = (0.0, 0.0, 10.0)
    direction: tuple = (0.0, 0.0, 1.0)
    up: tuple = (0.0, 1.0, 0.0)
    fov: float = float(F32(70.0) * (PI / F32(180.0)))  # 70f32.to_radians()

    @staticmethod
    def look_at(eye, center, up=(0.0, 1.0, 0.0), fov=None) -> "Camera":
        """Camera::look_at (camera.rs:53-66), evaluated in f32."""
        eye = np.asarray(eye, F32)
        center = np.asarray(center, F32)
        up = np.asarray(up, F32)
        d = center - eye
        d = d * (F32(1.0) / np.sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))
        k = (up[0] * d[0] + up[1] * d[1]) + up[2] * d[2]
        u = up - k * d
        u = u * (F32(1.0) / np.sqrt((u[0] * u[0] + u[1] * u[1]) + u[2] * u[2]))
        cam = Camera(tuple(map(float, eye)), tuple(map(float, d)), tuple(map(float, u)))
        if fov is not None:
            cam.fov = float(fov)
        return cam


@dataclass
class Octree:
    """new_octree::Octree (new_octree.rs:13-19) + leaf payload -> primitive lists."""
    octant_mask: np.ndarray      # uint16 [n]
    octant_children: np.ndarray  # uint32 [n, 8]
    root: int
    depth: int
    leaf_first: np.ndarray       # uint32 [leaves]
    leaf_count: np.ndarray       # uint32 [leaves]
    leaf_prims: np.ndarray       # uint32 [sum(count)]

    @property
    def scale(self) -> float:
        """Octree::scale (new_octree.rs:40-42)."""
        return float(np.exp2(-float(self.depth)))

    @property
    def octant_count(self) -> int:
        return int(self.octant_mask.shape[0])

    @staticmethod
    def empty(depth: int) -> "Octree":
        return Octree(np.zeros(1, np.uint16), np.zeros((1, 8), np.uint32), 0, depth,
                      np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32))

    def traversal_data(self, ray, max_dst: float = 1024.0, octants=None):
        """Octree::get_traversal_data (octree_traversal.rs:537-714) through liboctpt's host query:
        (start octant, scale, index_stack[24], time_stack[24]) for one ray (origin, direction).
        `octants` may pass a cached octants_struct() to skip its per-call conversion."""
        lib = _lib.load()
        arr = octants if octants is not None else self.octants_struct()
        r = np.ascontiguousarray(ray, F32).reshape(6)
        start, scale = C.c_uint32(), C.c_uint32()
        idx = np.zeros(24, np.uint32)
        ts = np.zeros(24, F32)
        st = lib.octpt_traversal_data(C.cast(arr, C.c_void_p), self.octant_count, self.root, self.depth,
                                      r.ctypes.data_as(C.c_void_p), max_dst, C.byref(start), C.byref(scale),
                                      idx.ctypes.data_as(C.c_void_p), ts.ctypes.data_as(C.c_void_p))
        _lib.check(lib, None, st)
        return start.value, scale.value, idx, ts

    def octants_struct(self):
        arr = (_lib.Octant * self.octant_count)()
        buf = np.frombuffer(arr, dtype=np.dtype([("m", "<u2"), ("r", "<u2"), ("c", "<u4", (8,))]))
        buf["m"] = self.octant_mask
        buf["r"] = 0
        buf["c"] = self.octant_children
        return arr


@dataclass
class Scene:
    """scene::Scene (scene/mod.rs:146-156): spheres and cuboids, plus block models:
    a cuboid whose cuboid_model entry is not MODEL_NONE is a block-model instance whose surface is
    the model's quads (Scene::quads, scene/mod.rs:153), as the reference's ResourceModel::Quad leaf."""
    spheres: np.ndarray = field(default_factory=lambda: np.zeros((0, 4), F32))          # cx, cy, cz, r
    sphere_material: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    cuboids: np.ndarray = field(default_factory=lambda: np.zeros((0, 6), F32))          # min xyz, max xyz
    cuboid_material: np.ndarray = field(default_factory=lambda: np.zeros((0, 6), np.uint32))
    materials: list = field(default_factory=lambda: [air_material()])
    textures: list = field(default_factory=lambda: [Texture()])
    sun: Sun = field(default_factory=Sun)
    strategy: SunSamplingStrategy = field(default_factory=lambda: STRATEGY_IMPORTANCE)
    emitters_enabled: bool = True
    cuboid_model: np.ndarray | None = None   # u32 per cuboid, _lib.MODEL_NONE = plain box
    models: np.ndarray = field(default_factory=lambda: np.zeros((0, 2), np.uint32))   # first quad, count
    quads: np.ndarray = field(default_factory=lambda: np.zeros(0, _lib.QUAD_DTYPE))
    f_sub_surface: float = 0.3  # Scene::f_sub_surface (scene/mod.rs:152), used by sun sampling (path_tracer.rs:240)
    octree: Octree | None = None
    # block-value leaves: the octree's leaf payloads are block ids into `blocks` (six face
    # materials per block, Face order W,E,Bottom,Top,South,North), block_model[b] = MODEL_NONE (the block
    # fills its leaf cell) or a block model; `cells` (n, 4) = (x, y, z, block) the builder voxelises
    blocks: np.ndarray | None = None
    block_model: np.ndarray | None = None
    cells: np.ndarray | None = None

    # ---------------------------------------------------------------- octree
    def build_octree(self, depth: int, renderer=None, compact: bool = False) -> Octree:
        """Voxelise the primitives with the product builder: octpt_build_octree (host), or with a
        HipRenderer given, octpt_build_octree_device on its GPU (the same arrays).  compact: merge
        eight sibling leaves holding the same primitive list, bottom-up (OCTPT_BUILD_COMPACT,
        Octant::is_compactable, new_octree.rs:227-233).  A block-value scene (C23) builds from its
        cells with octpt_build_block_octree (compact: eight equal block values merge)."""
        lib = _lib.load()
        if self.blocks is not None:
            return self._build_block_octree(lib, depth, compact)
        sph = self.sphere_structs()
        cub = self.cuboid_structs()
        handle = C.c_void_p()
        args = (C.cast(sph, C.c_void_p) if len(self.spheres) else None, len(self.spheres),
                C.cast(cub, C.c_void_p) if len(self.cuboids) else None, len(self.cuboids), depth,
                _lib.BUILD_COMPACT if compact else 0, C.byref(handle))
        if renderer is None:
            _lib.check(lib, None, lib.octpt_build_octree_ex(*args))
        else:
            _lib.check(lib, renderer._ctx, lib.octpt_build_octree_device_ex(renderer._ctx, *args))
        try:
            v = _lib.OctreeView()
            _lib.check(lib, None, lib.octpt_octree_get_view(handle, C.byref(v)))
            dt = np.dtype([("m", "<u2"), ("r", "<u2"), ("c", "<u4", (8,))])

            def view(ptr, nbytes):  # zero-copy view of library memory (copied out below)
                return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))

            oct_ = view(v.octants, 36 * v.octant_count).view(dt)

            def u32(ptr, n):
                return view(ptr, 4 * n).view(np.uint32).copy() if n else np.zeros(0, np.uint32)

            self.octree = Octree(oct_["m"].copy(), oct_["c"].copy(), int(v.root), int(v.depth),
                                 u32(v.leaf_first, v.leaf_table_size), u32(v.leaf_count, v.leaf_table_size),
                                 u32(v.leaf_prims, v.leaf_prim_count))
        finally:
            lib.octpt_octree_free(handle)
        return self.octree

    def _build_block_octree(self, lib, depth: int, compact: bool) -> Octree:
        cells = np.ascontiguousarray(self.cells, np.uint32).reshape(-1, 4)
        handle = C.c_void_p()
        _lib.check(lib, None, lib.octpt_build_block_octree(cells.ctypes.data_as(C.c_void_p) if len(cells) else None,
                                                           len(cells), depth, _lib.BUILD_COMPACT if compact else 0,
                                                           C.byref(handle)))
        try:
            v = _lib.OctreeView()
            _lib.check(lib, None, lib.octpt_octree_get_view(handle, C.byref(v)))
            dt = np.dtype([("m", "<u2"), ("r", "<u2"), ("c", "<u4", (8,))])
            raw = np.ctypeslib.as_array(C.cast(v.octants, C.POINTER(C.c_uint8)), shape=(36 * v.octant_count,))
            oct_ = raw.view(dt)
            z = np.zeros(0, np.uint32)
            self.octree = Octree(oct_["m"].copy(), oct_["c"].copy(), int(v.root), int(v.depth), z, z.copy(), z.copy())
        finally:
            lib.octpt_octree_free(handle)
        return self.octree

    def block_structs(self):
        """octpt_block rows of `blocks` / `block_model` (C23)."""
        n = len(self.blocks)
        arr = (_lib.Block * max(n, 1))()
        buf = np.frombuffer(arr, dtype=np.dtype([("f", "<u4", (6,)), ("m", "<u4"), ("r", "<u4")]))
        buf["f"][:n] = np.asarray(self.blocks, np.uint32).reshape(-1, 6)
        buf["m"][:n] = (self.block_model if self.block_model is not None
                        else np.full(n, _lib.MODEL_NONE, np.uint32))
        return arr

    # ---------------------------------------------------------------- ABI views
    def sphere_structs(self):
        n = len(self.spheres)
        arr = (_lib.Sphere * max(n, 1))()
        if n:
            buf = np.frombuffer(arr, dtype=np.dtype([("c", "<f4", (3,)), ("r", "<f4"), ("m", "<u4"), ("p", "<u4", (3,))]))
            buf["c"][:n] = self.spheres[:, :3]
            buf["r"][:n] = self.spheres[:, 3]
            buf["m"][:n] = self.sphere_material
        return arr

    def cuboid_structs(self):
        n = len(self.cuboids)
        arr = (_lib.Cuboid * max(n, 1))()
        if n:
            buf = np.frombuffer(arr, dtype=np.dtype([("lo", "<f4", (3,)), ("hi", "<f4", (3,)), ("m", "<u4", (6,))]))
            buf["lo"][:n] = self.cuboids[:, :3]
            buf["hi"][:n] = self.cuboids[:, 3:]
            buf["m"][:n] = self.cuboid_material
        return arr

    def sun_struct(self) -> "_lib.Sun":
        s = self.sun
        st = self.strategy
        return _lib.Sun(s.azimuth, s.altitude, s.radius, (C.c_float * 4)(*s.color), (C.c_float * 3)(*s.apparent_color),
                        int(s.draw_texture), int(s.texture_modification), s.importance_sample_chance,
                        s.importance_sample_radius, s.luminosity, (C.c_uint8 * 4)(*s.texture_rgba),
                        int(st.importance_sampling), int(st.diffuse_sun), int(st.sun_sampling),
                        int(st.strict_direct_light), int(st.sun_luminosity), s.luminosity_pdf)

    def to_desc(self, octree: bool = True, depth: int | None = None):
        """octpt_scene_desc for octpt_scene_upload; returns (desc, keepalive).  octree=False: the
        octree fields stay NULL / 0 and `depth` is the build depth (octpt_scene_build_device)."""
        if octree and self.octree is None:
            raise ValueError("scene has no octree: call build_octree(depth) first")
        t = self.octree
        keep = []

        def ptr(a):
            if a is None or (hasattr(a, "__len__") and len(a) == 0):
                return None
            keep.append(a)
            if isinstance(a, np.ndarray):
                return a.ctypes.data_as(C.c_void_p)
            return C.cast(a, C.c_void_p)

        if octree:
            octs = t.octants_struct()
            lf = np.ascontiguousarray(t.leaf_first, np.uint32)
            lc = np.ascontiguousarray(t.leaf_count, np.uint32)
            lp = np.ascontiguousarray(t.leaf_prims, np.uint32)
        mats = (_lib.Material * len(self.materials))(*[
            _lib.Material(m.ior, m.specular, m.emittance, m.roughness, m.metalness, m.texture_index, m.tint_index, m.flags)
            for m in self.materials])
        texs = (_lib.Texture * len(self.textures))()
        for i, tx in enumerate(self.textures):
            texs[i].kind = tx.kind
            texs[i].rgba[:] = list(tx.rgba)
            if tx.kind == _lib.TEXTURE_IMAGE:
                px = np.ascontiguousarray(tx.pixels, np.uint8)
                keep.append(px)
                texs[i].width, texs[i].height = px.shape[1], px.shape[0]
                texs[i].pixels = px.ctypes.data
        desc = _lib.SceneDesc()
        desc.abi_version = _lib.OCTPT_ABI_VERSION
        if octree:
            desc.octants = ptr(octs)
            desc.octant_count = t.octant_count
            desc.root = t.root
            desc.depth = t.depth
            desc.leaf_first = ptr(lf)
            desc.leaf_count = ptr(lc)
            desc.leaf_table_size = len(lf)
            desc.leaf_prims = ptr(lp)
            desc.leaf_prim_count = len(lp)
            keep.append(octs)
        else:
            desc.depth = int(depth if depth is not None else (t.depth if t is not None else 0))
        desc.spheres = ptr(self.sphere_structs()) if len(self.spheres) else None
        desc.sphere_count = len(self.spheres)
        desc.cuboids = ptr(self.cuboid_structs()) if len(self.cuboids) else None
        desc.cuboid_count = len(self.cuboids)
        desc.materials = ptr(mats)
        desc.material_count = len(self.materials)
        desc.textures = ptr(texs)
        desc.texture_count = len(self.textures)
        desc.sun = self.sun_struct()
        desc.emitters_enabled = int(self.emitters_enabled)
        desc.f_sub_surface = self.f_sub_surface
        if (self.cuboid_model is not None and len(self.cuboids)) or self.blocks is not None:
            mdl = np.zeros((max(len(self.models), 1), 4), np.uint32)
            mdl[: len(self.models), 1:3] = np.asarray(self.models, np.uint32).reshape(-1, 2)
            qd = np.ascontiguousarray(self.quads)
            if self.cuboid_model is not None and len(self.cuboids):
                desc.cuboid_model = ptr(np.ascontiguousarray(self.cuboid_model, np.uint32))
            desc.models = ptr(mdl) if len(self.models) else None
            desc.model_count = len(self.models)
            desc.quads = ptr(qd) if len(qd) else None
            desc.quad_count = len(qd)
        if self.blocks is not None:  # block-value leaves (C23)
            desc.blocks = ptr(self.block_structs())
            desc.block_count = len(self.blocks)
        keep.extend([mats, texs])
        return desc, keep


@dataclass
class RenderSettings:
    width: int
    height: int
    spp: int
    max_depth: int = 5       # path_tracer.rs:56
    seed: int = 1
    branch_count: int = 1    # SURVEY contract C6


# ------------------------------------------------------------------------------
# seeded synthetic scene generator (integer hash -> f32, identical on every machine)
# ------------------------------------------------------------------------------
def _lowbias32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32)
    with np.errstate(over="ignore"):
        x ^= x >> np.uint32(16)
        x *= np.uint32(0x7FEB352D)
        x ^= x >> np.uint32(15)
        x *= np.uint32(0x846CA68B)
        x ^= x >> np.uint32(16)
    return x


def scene_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n uniform f32 in [0,1) for (seed, stream): (lowbias32(key ^ i) >> 8) * 2^-24."""
    key = _lowbias32(np.array([(seed * 0x9E3779B9 + stream * 0x85EBCA6B) & 0xFFFFFFFF], np.uint32))[0]
    i = np.arange(n, dtype=np.uint32)
    h = _lowbias32(i ^ key)
    return (h >> np.uint32(8)).astype(F32) * F32(1.0 / 16777216.0)


def _uniform_range(seed, stream, n, lo, hi):
    u = scene_uniform(seed, stream, n)
    return F32(lo) + (F32(hi) - F32(lo)) * u


DIFFUSE_PALETTE = [(200, 60, 50), (60, 170, 80), (70, 90, 210), (220, 200, 70), (180, 180, 180), (230, 120, 40),
                   (140, 70, 180), (90, 200, 200)]


def primitive_materials(scene: Scene) -> dict:
    """Standard material set: 8 diffuse colours, metal, glossy, glass (+ air at index 0)."""
    scene.textures = [Texture()]  # index 0: DEFAULT_TEXTURE for air
    scene.materials = [air_material(0)]
    ids = {"diffuse": []}
    for rgb in DIFFUSE_PALETTE:
        scene.textures.append(Texture.color(*rgb))
        scene.materials.append(Material(texture_index=len(scene.textures) - 1))
        ids["diffuse"].append(len(scene.materials) - 1)
    scene.textures.append(Texture.color(230, 230, 235))
    scene.materials.append(Material(metalness=1.0, roughness=0.1, texture_index=len(scene.textures) - 1))
    ids["metal"] = len(scene.materials) - 1
    scene.textures.append(Texture.color(240, 240, 240))
    scene.materials.append(Material(specular=0.3, roughness=0.05, texture_index=len(scene.textures) - 1))
    ids["glossy"] = len(scene.materials) - 1
    scene.textures.append(Texture.color(255, 255, 255, 0))
    scene.materials.append(Material(ior=1.5, flags=REFRACTIVE, texture_index=len(scene.textures) - 1))
    ids["glass"] = len(scene.materials) - 1
    return ids


def procedural_terrain(seed: int, w: int = 1024, h: int = 512) -> np.ndarray:
    """Deterministic stand-in for a photographic colour map: bilinear value noise (4 octaves)
    mapped to water / land / rock / snow colours, RGBA8, opaque."""
    acc = np.zeros((h, w), np.float32)
    for o, (gx, gy) in enumerate([(8, 4), (16, 8), (32, 16), (64, 32)]):
        g = scene_uniform(seed, 100 + o, (gy + 1) * (gx + 1)).reshape(gy + 1, gx + 1)
        ys = np.linspace(0, gy, h, endpoint=False, dtype=np.float32)
        xs = np.linspace(0, gx, w, endpoint=False, dtype=np.float32)
        y0, x0 = ys.astype(np.int64), xs.astype(np.int64)
        fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
        v = (g[y0][:, x0] * (1 - fx) + g[y0][:, x0 + 1] * fx) * (1 - fy) + \
            (g[y0 + 1][:, x0] * (1 - fx) + g[y0 + 1][:, x0 + 1] * fx) * fy
        acc += v / (2 ** o)
    acc /= acc.max()
    pal = np.array([(20, 40, 120), (30, 90, 170), (60, 140, 60), (120, 110, 60), (150, 140, 130), (240, 240, 245)],
                   np.float32)
    stops = np.array([0.0, 0.45, 0.5, 0.65, 0.8, 1.0], np.float32)
    rgb = np.stack([np.interp(acc, stops, pal[:, c]) for c in range(3)], -1)
    out = np.empty((h, w, 4), np.uint8)
    out[..., :3] = np.clip(rgb, 0, 255).astype(np.uint8)
    out[..., 3] = 255
    return out


def procedural_atlas(seed: int, tiles: int = 16, tile: int = 16) -> np.ndarray:
    """A 16x16 atlas of 16x16-texel tiles (block-texture layout) with per-tile colour and texel
    noise; about 2 % of the texels are fully transparent (alpha 0: the transparent-texel path, C4)."""
    n = tiles * tile
    base = (scene_uniform(seed, 200, tiles * tiles * 3).reshape(tiles, tiles, 3) * 200 + 40)
    noise = scene_uniform(seed, 201, n * n).reshape(n, n) * 40 - 20
    rgb = np.repeat(np.repeat(base, tile, 0), tile, 1) + noise[..., None]
    out = np.empty((n, n, 4), np.uint8)
    out[..., :3] = np.clip(rgb, 0, 255).astype(np.uint8)
    out[..., 3] = np.where(scene_uniform(seed, 202, n * n).reshape(n, n) < 0.02, 0, 255).astype(np.uint8)
    return out


C4_TEXTURES = Path(__file__).resolve().parent / "assets" / "c4_textures.npz"


def c4_textures() -> tuple:
    """(earthmap, greasy): the reference's test_assets/earthmap.jpg (1024x512) and greasy.jpg (3024x4032, box-
    averaged by 8 to 378x504) as RGBA8 with alpha 255, as RTWImage widens 3-channel images (rtw_image.rs:79-84);
    decoded once by tools/make_c4_assets.py, the fixture ships in the package (no JPEG decode on the GPU path)."""
    with np.load(C4_TEXTURES) as z:
        return z["earthmap"], z["greasy"]


def textured_materials(scene: Scene, seed: int) -> dict:
    """primitive_materials with the diffuse set replaced by image-textured materials (C4, SURVEY.md §8d: the
    reference's own earthmap and a downsampled greasy, c4_textures; round 4 and before used the procedural
    stand-ins procedural_terrain / procedural_atlas)."""
    ids = primitive_materials(scene)
    earth, greasy = c4_textures()
    scene.textures.append(Texture.image(earth))
    scene.materials.append(Material(texture_index=len(scene.textures) - 1))
    terrain = len(scene.materials) - 1
    scene.textures.append(Texture.image(greasy))
    scene.materials.append(Material(texture_index=len(scene.textures) - 1))
    atlas = len(scene.materials) - 1
    ids["diffuse"] = [terrain, atlas]
    return ids


def _value_noise(seed: int, stream: int, h: int, w: int, grids) -> np.ndarray:
    """Bilinear value noise, octaves with the given (gx, gy) lattice sizes, normalised to [0, 1]."""
    acc = np.zeros((h, w), np.float32)
    for o, (gx, gy) in enumerate(grids):
        g = scene_uniform(seed, stream + o, (gy + 1) * (gx + 1)).reshape(gy + 1, gx + 1)
        ys = np.linspace(0, gy, h, endpoint=False, dtype=np.float32)
        xs = np.linspace(0, gx, w, endpoint=False, dtype=np.float32)
        y0, x0 = ys.astype(np.int64), xs.astype(np.int64)
        fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
        acc += ((g[y0][:, x0] * (1 - fx) + g[y0][:, x0 + 1] * fx) * (1 - fy) +
                (g[y0 + 1][:, x0] * (1 - fx) + g[y0 + 1][:, x0 + 1] * fx) * fy) / (2 ** o)
    acc -= acc.min()
    return acc / acc.max()


BLOCK_TILES = {  # base colour, texel noise amplitude, (top rows colour, rows) for side tiles
    "grass_top": ((95, 159, 53), 30, None), "grass_side": ((134, 96, 67), 24, ((95, 159, 53), 4)),
    "dirt": ((134, 96, 67), 24, None), "stone": ((125, 125, 125), 30, None),
    "snow": ((240, 244, 250), 10, None), "snow_side": ((134, 96, 67), 24, ((240, 244, 250), 5)),
    "sand": ((219, 207, 163), 18, None),
}


def block_tile(seed: int, stream: int, base, amp, top=None) -> np.ndarray:
    """A 16x16 RGBA8 block texture: base colour + per-texel noise, optionally a differently
    coloured top band (side faces of grass / snow blocks)."""
    noise = scene_uniform(seed, stream, 256).reshape(16, 16) * (2 * amp) - amp
    rgb = np.broadcast_to(np.float32(base), (16, 16, 3)).copy()
    if top is not None:
        rgb[: top[1]] = np.float32(top[0])
    out = np.empty((16, 16, 4), np.uint8)
    out[..., :3] = np.clip(rgb + noise[..., None], 0, 255).astype(np.uint8)
    out[..., 3] = 255
    return out


def block_materials(scene: Scene, seed: int) -> dict:
    """Register the BLOCK_TILES textures / materials; returns tile name -> material index."""
    if not scene.textures:
        scene.textures = [Texture()]
        scene.materials = [air_material(0)]
    mat = {}
    for k, (name, (base, amp, top)) in enumerate(BLOCK_TILES.items()):
        scene.textures.append(Texture.image(block_tile(seed, 300 + k, base, amp, top)))
        scene.materials.append(Material(texture_index=len(scene.textures) - 1))
        mat[name] = len(scene.materials) - 1
    return mat


def voxel_terrain(scene: Scene, seed: int, side: int, origin: int = 24):
    """C5's voxel world: a value-noise heightmap over side x side columns starting
    at (origin, origin), heights in [48, 176); every column holds its top block plus the blocks a
    lower neighbour exposes, all unit cubes [x, x+1)^3 (one octree cell each).
    Faces W, E, Bottom, Top, South, North take materials of 16x16 block textures by block kind:
    sand below 64, snow from 150, grass otherwise; exposed blocks below the top are dirt (3 deep)
    then stone.  Returns (cuboids [n, 6], face materials [n, 6])."""
    mat = block_materials(scene, seed)
    # face order W, E, Bottom, Top, South, North (cuboid.rs:9-29)
    kinds = np.array([[mat["grass_side"]] * 2 + [mat["dirt"], mat["grass_top"]] + [mat["grass_side"]] * 2,
                      [mat["dirt"]] * 6, [mat["stone"]] * 6,
                      [mat["snow_side"]] * 2 + [mat["dirt"], mat["snow"]] + [mat["snow_side"]] * 2,
                      [mat["sand"]] * 6], np.uint32)
    hmap = (48 + np.floor(128 * _value_noise(seed, 400, side, side, [(6, 6), (12, 12), (24, 24), (48, 48)])))
    h = hmap.astype(np.int64)
    pad = np.pad(h, 1, mode="edge")
    nbr = np.minimum.reduce([pad[:-2, 1:-1], pad[2:, 1:-1], pad[1:-1, :-2], pad[1:-1, 2:]])
    lo = np.minimum(h, nbr + 1)  # lowest exposed block of the column
    count = (h - lo + 1).ravel()
    zz, xx = np.meshgrid(np.arange(side), np.arange(side), indexing="ij")
    col = np.repeat(np.arange(side * side), count)
    first = np.repeat(np.cumsum(count) - count, count)
    top = h.ravel()[col]
    y = top - (np.arange(len(col)) - first)
    below = top - y
    kind = np.where(below >= 4, 2, np.where(below >= 1, 1, np.where(top >= 150, 3, np.where(top < 64, 4, 0))))
    x = xx.ravel()[col] + origin
    z = zz.ravel()[col] + origin
    lo3 = np.stack([x, y, z], 1).astype(F32)
    return np.concatenate([lo3, lo3 + F32(1.0)], 1), kinds[kind]


# ---------------------------------------------------------------------------- block models (C19)
# Face order of the reference's block-model Cuboid (resource_manager.rs:583-588).
MODEL_FACES = ("west", "east", "down", "up", "north", "south")


def _rotation(axis: str, angle_deg: float) -> np.ndarray:
    a = np.float32(np.deg2rad(angle_deg))
    c, s = np.float32(np.cos(a)), np.float32(np.sin(a))
    if axis == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]], F32)
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]], F32)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], F32)


def element_quads(frm, to, faces: dict, rotation=None) -> list:
    """One Minecraft block-model element (from / to in 1/16 block) -> voxel-local quad rows: the
    per-face origin / u / v of Quad::from_face_name (quad.rs:26-68, the commented-out body), the
    face uv rectangle / 16 as texture ranges, and an optional element rotation (origin in 1/16,
    axis, degrees) applied as Quad::transform_about_pivot (quad.rs:115-125).
    faces: name -> material or (material, (u1, v1, u2, v2))."""
    f = np.asarray(frm, F32) / F32(16.0)
    t = np.asarray(to, F32) / F32(16.0)
    geo = {
        "down": ((f[0], f[1], f[2]), (t[0] - f[0], 0, 0), (0, 0, t[2] - f[2])),
        "up": ((t[0], t[1], f[2]), (f[0] - t[0], 0, 0), (0, 0, t[2] - f[2])),
        "north": ((t[0], f[1], f[2]), (f[0] - t[0], 0, 0), (0, t[1] - f[1], 0)),
        "south": ((f[0], f[1], t[2]), (t[0] - f[0], 0, 0), (0, t[1] - f[1], 0)),
        "west": ((f[0], f[1], f[2]), (0, 0, t[2] - f[2]), (0, t[1] - f[1], 0)),
        "east": ((t[0], f[1], t[2]), (0, 0, f[2] - t[2]), (0, t[1] - f[1], 0)),
    }
    rows = []
    for name in MODEL_FACES:
        if name not in faces:
            continue
        spec = faces[name]
        mat, uv = (spec, (0.0, 0.0, 16.0, 16.0)) if np.isscalar(spec) else spec
        o, u, v = (np.asarray(x, F32) for x in geo[name])
        if rotation is not None:
            piv = np.asarray(rotation[0], F32) / F32(16.0)
            m = _rotation(rotation[1], rotation[2])
            o = (m @ (o - piv)).astype(F32) + piv
            u = (m @ u).astype(F32)
            v = (m @ v).astype(F32)
        uv = np.asarray(uv, F32) / F32(16.0)
        rows.append((o, int(mat), u, v, (uv[0], uv[2]), (uv[1], uv[3]), (0, 0)))
    return rows


def alpha_tile(seed: int, stream: int, base, amp, mask: np.ndarray) -> np.ndarray:
    """block_tile with alpha 0 where mask is False (plants, glass panes: transparent texels)."""
    out = block_tile(seed, stream, base, amp)
    out[..., 3] = np.where(mask, 255, 0).astype(np.uint8)
    return out


def block_models(scene: Scene, seed: int) -> dict:
    """A small Minecraft-style block-model set: slab, stairs, cross plant, fence
    post, tilted torch and glass pane.  Appends their textures, materials, quads and models to the
    scene and returns name -> model index."""
    def tile(name, img):
        scene.textures.append(Texture.image(img))
        scene.materials.append(Material(texture_index=len(scene.textures) - 1))
        return len(scene.materials) - 1

    planks = tile("planks", block_tile(seed, 350, (162, 130, 78), 20))
    blades = scene_uniform(seed, 351, 256).reshape(16, 16) < 0.45
    blades[:, ::3] = False
    plant = tile("plant", alpha_tile(seed, 352, (70, 150, 40), 30, blades))
    torch = tile("torch", block_tile(seed, 353, (120, 90, 40), 20, ((255, 210, 90), 3)))
    frame = np.zeros((16, 16), bool)
    frame[[0, 15], :] = frame[:, [0, 15]] = True
    glass = tile("glass", alpha_tile(seed, 354, (200, 225, 235), 10, frame))
    all6 = lambda m: {k: m for k in MODEL_FACES}  # noqa: E731
    defs = {
        "slab": [element_quads((0, 0, 0), (16, 8, 16), {**all6(planks), **{k: (planks, (0, 8, 16, 16)) for k in
                                                                           ("west", "east", "north", "south")}})],
        "stairs": [element_quads((0, 0, 0), (16, 8, 16), all6(planks)),
                   element_quads((8, 8, 0), (16, 16, 16), all6(planks))],
        "plant": [element_quads((0.8, 0, 8), (15.2, 16, 8), {"north": plant, "south": plant}, ((8, 8, 8), "y", 45.0)),
                  element_quads((8, 0, 0.8), (8, 16, 15.2), {"west": plant, "east": plant}, ((8, 8, 8), "y", 45.0))],
        "post": [element_quads((6, 0, 6), (10, 16, 10), all6(planks))],
        "torch": [element_quads((7, 0, 7), (9, 10, 9), all6(torch), ((8, 0, 8), "x", -22.5))],
        "pane": [element_quads((7, 0, 0), (9, 16, 16), all6(glass))],
    }
    rows, models, ids = [], [], {}
    for name, elems in defs.items():
        quads = [q for e in elems for q in e]
        ids[name] = len(models)
        models.append((len(rows), len(quads)))
        rows.extend(quads)
    base = len(scene.quads)
    q = np.zeros(len(rows), _lib.QUAD_DTYPE)
    for i, (o, m, u, v, tu, tv, _) in enumerate(rows):
        q[i] = (o, m, u, v, tu, tv, (0, 0))
    scene.quads = np.concatenate([scene.quads, q])
    mb = len(scene.models)
    scene.models = np.concatenate([np.asarray(scene.models, np.uint32).reshape(-1, 2),
                                   np.array([(base + a, n) for a, n in models], np.uint32).reshape(-1, 2)])
    return {k: mb + v for k, v in ids.items()}


def place_models(scene: Scene, seed: int, ids: dict, positions: np.ndarray, stream: int = 360):
    """Append block-model instances (unit-voxel cuboids with a cuboid_model entry) at integer
    voxel positions [n, 3]; the model per position is drawn from `ids` with plants most likely."""
    n = len(positions)
    names = list(ids)
    weights = np.array([0.10 if k != "plant" else 0.50 for k in names], np.float64)
    cdf = np.cumsum(weights / weights.sum())
    pick = np.searchsorted(cdf, scene_uniform(seed, stream, n).astype(np.float64), side="right")
    model = np.array([ids[names[min(i, len(names) - 1)]] for i in pick], np.uint32)
    lo = np.asarray(positions, F32)
    box = np.concatenate([lo, lo + F32(1.0)], 1)
    old = len(scene.cuboids)
    cm = scene.cuboid_model if scene.cuboid_model is not None else np.full(old, _lib.MODEL_NONE, np.uint32)
    scene.cuboids = np.concatenate([scene.cuboids.reshape(-1, 6), box]).astype(F32)
    fm = np.zeros((n, 6), np.uint32)  # unused by model instances; any valid material
    scene.cuboid_material = np.concatenate([scene.cuboid_material.reshape(-1, 6), fm]).astype(np.uint32)
    scene.cuboid_model = np.concatenate([cm, model]).astype(np.uint32)


def voxel_blocks(scene: Scene, seed: int, positions: np.ndarray):
    """Grass blocks (voxel_terrain's textures) at integer positions [n, 3]: (cuboids, face materials)."""
    m = block_materials(scene, seed)
    face = np.array([m["grass_side"]] * 2 + [m["dirt"], m["grass_top"]] + [m["grass_side"]] * 2, np.uint32)
    lo = np.asarray(positions, F32)
    return np.concatenate([lo, lo + F32(1.0)], 1), np.tile(face, (len(lo), 1))


def terrain_tops(seed: int, side: int, origin: int = 24) -> np.ndarray:
    """The top block of every voxel_terrain column, [side * side, 3] integer (x, y, z)."""
    hmap = (48 + np.floor(128 * _value_noise(seed, 400, side, side, [(6, 6), (12, 12), (24, 24), (48, 48)])))
    zz, xx = np.meshgrid(np.arange(side), np.arange(side), indexing="ij")
    return np.stack([xx.ravel() + origin, hmap.astype(np.int64).ravel(), zz.ravel() + origin], 1)


def voxels_to_blocks(scene: Scene) -> Scene:
    """The same world with block-value leaves, the reference's own leaf form: every
    unit-voxel cuboid [x, x+1)^3 becomes a cell whose leaf value is a block id; blocks are the distinct
    (six face materials, block model) rows.  Materials, textures, models, quads, sun and strategy are
    shared with `scene`; the octree is built by build_octree (octpt_build_block_octree)."""
    cub = np.asarray(scene.cuboids, F32).reshape(-1, 6)
    lo = cub[:, :3]
    if not (np.all(cub[:, 3:] == lo + F32(1.0)) and np.all(lo == np.floor(lo)) and np.all(lo >= 0)):
        raise ValueError("voxels_to_blocks: every cuboid must be a unit voxel [x, x+1)^3 at integer x >= 0")
    model = (np.asarray(scene.cuboid_model, np.uint32) if scene.cuboid_model is not None
             else np.full(len(cub), _lib.MODEL_NONE, np.uint32))
    fm = np.asarray(scene.cuboid_material, np.uint32).reshape(-1, 6).copy()
    fm[model != _lib.MODEL_NONE] = 0  # a model block's faces come from its quads
    rows = np.concatenate([fm, model[:, None]], 1)
    table, inv = np.unique(rows, axis=0, return_inverse=True)
    out = Scene(materials=scene.materials, textures=scene.textures, sun=scene.sun, strategy=scene.strategy,
                emitters_enabled=scene.emitters_enabled, models=scene.models, quads=scene.quads,
                f_sub_surface=scene.f_sub_surface)
    out.blocks = np.ascontiguousarray(table[:, :6], np.uint32)
    out.block_model = np.ascontiguousarray(table[:, 6], np.uint32)
    out.cells = np.concatenate([lo.astype(np.uint32), inv.reshape(-1, 1).astype(np.uint32)], 1)
    return out


def solid_terrain(scene: Scene, seed: int, side: int, origin: int = 24, floor: int = 0):
    """A block-value world on voxel_terrain's heightmap, every column solid from `floor`
    to its top -- the shape of a Minecraft region, whose underground compacts into LOD leaves (the
    section builder's Lod(section_fill_block) and RegionOctreeBuilder's Lod(data), new_octree.rs:534-537,
    586, 727).  Blocks: 0 grass, 1 dirt, 2 stone, 3 snow, 4 sand (voxel_terrain's face materials); the top
    block by height as there, three dirt below it, stone beneath.  Sets scene.blocks / cells."""
    mat = block_materials(scene, seed)
    scene.blocks = np.array([[mat["grass_side"]] * 2 + [mat["dirt"], mat["grass_top"]] + [mat["grass_side"]] * 2,
                             [mat["dirt"]] * 6, [mat["stone"]] * 6,
                             [mat["snow_side"]] * 2 + [mat["dirt"], mat["snow"]] + [mat["snow_side"]] * 2,
                             [mat["sand"]] * 6], np.uint32)
    scene.block_model = np.full(5, _lib.MODEL_NONE, np.uint32)
    h = (48 + np.floor(128 * _value_noise(seed, 400, side, side, [(6, 6), (12, 12), (24, 24), (48, 48)]))).astype(
        np.int64).ravel()
    count = h - floor + 1
    col = np.repeat(np.arange(side * side, dtype=np.int64), count)
    first = np.repeat(np.cumsum(count) - count, count)
    below = np.arange(len(col), dtype=np.int64) - first  # 0 = the top block
    top = h[col]
    kind = np.where(below >= 4, 2, np.where(below >= 1, 1, np.where(top >= 150, 3, np.where(top < 64, 4, 0))))
    cells = np.empty((len(col), 4), np.uint32)
    cells[:, 0] = col % side + origin
    cells[:, 1] = top - below
    cells[:, 2] = col // side + origin
    cells[:, 3] = kind
    scene.cells = cells
    return scene


def _assign_materials(ids, seed, n, stream=7):
    """70% diffuse, 15% metal, 10% glossy, 5% glass."""
    u = scene_uniform(seed, stream, n)
    pick = scene_uniform(seed, stream + 1, n)
    mats = np.empty(n, np.uint32)
    d = np.array(ids["diffuse"], np.uint32)
    mats[:] = d[np.minimum((pick * len(d)).astype(np.int64), len(d) - 1)]
    mats[(u >= 0.70) & (u < 0.85)] = ids["metal"]
    mats[(u >= 0.85) & (u < 0.95)] = ids["glossy"]
    mats[u >= 0.95] = ids["glass"]
    return mats


def random_spheres(seed: int, n: int, world: float, rmin: float, rmax: float):
    c = np.stack([_uniform_range(seed, 1 + a, n, 0.0, world) for a in range(3)], axis=1)
    r = _uniform_range(seed, 4, n, rmin, rmax)
    return np.concatenate([c, r[:, None]], axis=1).astype(F32)


def random_cuboids(seed: int, n: int, world: float, emin: float, emax: float):
    lo = np.stack([_uniform_range(seed, 11 + a, n, 0.0, world) for a in range(3)], axis=1)
    ext = np.stack([_uniform_range(seed, 14 + a, n, emin, emax) for a in range(3)], axis=1)
    return np.concatenate([lo, np.minimum(lo + ext, F32(world - 0.001))], axis=1).astype(F32)


CONFIGS = ("C1", "C1-as-is", "C2", "C3", "C4", "C5", "tiny", "blocks", "C3-in", "C5-fp", "C5b", "C5b-fp", "blocks-b",
           "C5s", "C5s-fp", "C5s-small", "cap")


def step_cap_world(scene: Scene, seed: int, floor_len: int = 1024, floor_w: int = 64, wall_x: int = 600):
    """A block-value world whose near-horizontal camera rays reach the reference's ESVO step
    cap (OCTREE_MAX_STEPS = 1000, octree_traversal.rs:13, 127) and miss: a checkerboard floor of blocks at
    y = 0 (every level-1 octant along the floor is present, so a ray skimming over it at 1 < y < 2 spends
    ~2 iterations per unit of distance without meeting a leaf), a stone wall at x = wall_x that only a
    walk counting fewer iterations than the reference would reach, and a picket of stone posts at x = 0,
    y = 1 (every fourth z): a camera tile whose pyramid grazes a post starts its rays right there, with a
    small bound of skipped iterations, and those of its rays that pass the post run into the cap after the
    start (the restart of a beam-started ray).  Sets scene.blocks / cells."""
    mat = block_materials(scene, seed)
    scene.blocks = np.array([[mat["grass_side"]] * 2 + [mat["dirt"], mat["grass_top"]] + [mat["grass_side"]] * 2,
                             [mat["stone"]] * 6], np.uint32)
    scene.block_model = np.full(2, _lib.MODEL_NONE, np.uint32)
    xx, zz = np.meshgrid(np.arange(floor_len), np.arange(floor_w), indexing="ij")
    keep = ((xx + zz) % 2 == 0) & ((xx < wall_x) | (xx >= wall_x + 4))
    floor = np.stack([xx[keep], np.zeros(keep.sum(), np.int64), zz[keep], np.zeros(keep.sum(), np.int64)], 1)
    wx, wy, wz = np.meshgrid(np.arange(wall_x, wall_x + 4), np.arange(8), np.arange(floor_w), indexing="ij")
    wall = np.stack([wx.ravel(), wy.ravel(), wz.ravel(), np.ones(wx.size, np.int64)], 1)
    pz = np.arange(0, floor_w, 4)
    posts = np.stack([np.zeros_like(pz), np.ones_like(pz), pz, np.ones_like(pz)], 1)
    scene.cells = np.concatenate([floor, wall, posts]).astype(np.uint32)
    return scene


C5_SIDE = 1000  # columns per side: 1,001,225 unit blocks with the exposed-side fill


def make_config(name: str, *, seed: int = 1, build: bool = True):
    """(Scene, Camera, RenderSettings) for BASELINE.json's configs.  A "b" suffix
    (C5b, C5b-fp, blocks-b) is the same voxel world with block-value leaves."""
    if name in ("C5b", "C5b-fp", "blocks-b"):
        base = {"C5b": "C5", "C5b-fp": "C5-fp", "blocks-b": "blocks"}[name]
        sc, cam, rs = make_config(base, seed=seed, build=False)
        sb = voxels_to_blocks(sc)
        depth = sc._depth  # type: ignore[attr-defined]
        if build:
            sb.build_octree(depth)
        else:
            sb._depth = depth  # type: ignore[attr-defined]
        return sb, cam, rs
    if name in ("C5s", "C5s-fp", "C5s-small"):
        # C5's heightmap as a solid block-value world (C23); C5s-small: 128 x 128 columns (tests)
        sc = Scene()
        side = 128 if name == "C5s-small" else C5_SIDE
        solid_terrain(sc, seed, side)
        depth = 11
        mid = 24 + side / 2
        cam = Camera.look_at((mid, 230.0, 24.0 - 60.0 * side / C5_SIDE), (mid, 100.0, mid))
        if name == "C5s-fp":
            cam = Camera.look_at((300.5, 190.0, 300.5), (800.0, 120.0, 800.0))
        rs = RenderSettings(3840, 2160, 1024, seed=seed)
        if build:
            sc.build_octree(depth)
        else:
            sc._depth = depth  # type: ignore[attr-defined]
        return sc, cam, rs
    if name == "cap":
        # camera rays that reach the reference's step cap (the beam start's iteration bound):
        # a wide, 8-row image at the horizon over step_cap_world's floor
        sc = Scene()
        step_cap_world(sc, seed)
        cam = Camera(eye=(-20.0, 1.5, 31.7), direction=(1.0, 0.0, 0.0), up=(0.0, 1.0, 0.0))
        rs = RenderSettings(4096, 8, 1, max_depth=2, seed=seed)
        if build:
            sc.build_octree(10)
        else:
            sc._depth = 10  # type: ignore[attr-defined]
        return sc, cam, rs
    sc = Scene()
    if name in ("C1", "C1-as-is"):
        ids = primitive_materials(sc)
        depth = 6
        sc.spheres = np.array([[32.0, 32.0, 32.0, 4.0]], F32)
        sc.sphere_material = np.array([ids["diffuse"][0]], np.uint32)
        cam = Camera(eye=(32.0, 32.0, 8.0), direction=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0))
        rs = RenderSettings(256, 256, 1, max_depth=1, seed=seed)
        if name == "C1-as-is":  # Scene::hit stubbed to false (scene/mod.rs:172-187): sky + sun only
            sc.octree = Octree.empty(depth)
            return sc, cam, rs
    elif name == "tiny":
        ids = primitive_materials(sc)
        depth = 5
        sc.spheres = random_spheres(seed, 40, 32.0, 0.5, 3.0)
        sc.sphere_material = _assign_materials(ids, seed, 40)
        sc.cuboids = random_cuboids(seed, 6, 32.0, 1.0, 4.0)
        cm = _assign_materials(ids, seed + 5, 6 * 6, stream=21).reshape(6, 6)
        sc.cuboid_material = cm
        cam = Camera.look_at((16.0, 20.0, -14.0), (16.0, 16.0, 16.0))
        rs = RenderSettings(64, 48, 4, seed=seed)
    elif name == "blocks":
        # block-model test world: a 24 x 24 floor of grass blocks with every model
        # of block_models() on it, close up
        depth = 5
        floor = np.stack(np.meshgrid(np.arange(4, 28), np.arange(4, 28), indexing="ij"), -1).reshape(-1, 2)
        pos = np.stack([floor[:, 0], np.full(len(floor), 8), floor[:, 1]], 1)
        sc.cuboids, sc.cuboid_material = voxel_blocks(sc, seed, pos)
        ids_m = block_models(sc, seed)
        on = pos[(pos[:, 0] + 2 * pos[:, 2]) % 3 == 0] + np.array([0, 1, 0])
        place_models(sc, seed, ids_m, on)
        cam = Camera.look_at((6.0, 16.0, -4.0), (16.0, 9.0, 16.0))
        rs = RenderSettings(64, 48, 4, seed=seed)
    elif name == "C2":
        ids = primitive_materials(sc)
        depth = 6
        sc.spheres = random_spheres(seed, 100, 64.0, 0.5, 3.0)
        sc.sphere_material = _assign_materials(ids, seed, 100)
        cam = Camera.look_at((32.0, 38.0, -28.0), (32.0, 32.0, 32.0))
        rs = RenderSettings(1280, 720, 64, seed=seed)
    elif name in ("C3", "C3-in"):
        ids = primitive_materials(sc)
        depth = 8
        sc.spheres = random_spheres(seed, 10_000, 256.0, 0.5, 2.5)
        sc.sphere_material = _assign_materials(ids, seed, 10_000)
        cam = Camera.look_at((128.0, 150.0, -110.0), (128.0, 128.0, 128.0))
        if name == "C3-in":  # camera inside the sphere cloud (the start chain's case)
            cam = Camera.look_at((128.3, 128.7, 127.6), (200.0, 140.0, 60.0))
        rs = RenderSettings(1920, 1080, 256, seed=seed)
    elif name == "C4":
        ids = textured_materials(sc, seed)
        depth = 10
        n = 50_000
        sc.spheres = random_spheres(seed, n, 1024.0, 0.5, 4.0)
        sc.sphere_material = _assign_materials(ids, seed, n)
        sc.cuboids = random_cuboids(seed, n, 1024.0, 0.5, 4.0)
        sc.cuboid_material = _assign_materials(ids, seed + 5, 6 * n, stream=21).reshape(n, 6)
        cam = Camera.look_at((512.0, 600.0, -420.0), (512.0, 512.0, 512.0))
        rs = RenderSettings(3840, 2160, 512, seed=seed)
    elif name in ("C5", "C5-fp"):
        depth = 11
        sc.cuboids, sc.cuboid_material = voxel_terrain(sc, seed, C5_SIDE)
        # block models (§8f row 1, C19) on 3 % of the grass / sand surface columns
        ids_m = block_models(sc, seed)
        tops = terrain_tops(seed, C5_SIDE)
        keep = (scene_uniform(seed, 361, len(tops)) < 0.03) & (tops[:, 1] < 150)
        place_models(sc, seed, ids_m, tops[keep] + np.array([0, 1, 0]))
        mid = 24 + C5_SIDE / 2
        cam = Camera.look_at((mid, 230.0, 24.0 - 60.0), (mid, 100.0, mid))
        if name == "C5-fp":  # first-person view inside the world above the terrain (heights < 176)
            cam = Camera.look_at((300.5, 190.0, 300.5), (800.0, 120.0, 800.0))
        rs = RenderSettings(3840, 2160, 1024, seed=seed)
    else:
        raise ValueError(f"unknown config {name!r}; known: {CONFIGS}")
    if build:
        sc.build_octree(depth)
    else:
        sc.octree = None
        sc._depth = depth  # type: ignore[attr-defined]
    return sc, cam, rs


def load_rgba_fixture(path: str | Path, width: int, height: int) -> np.ndarray:
    data = np.fromfile(path, dtype=np.uint8)
    return data.reshape(height, width, 4)
