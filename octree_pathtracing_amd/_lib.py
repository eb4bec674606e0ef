"""ctypes binding of liboctpt.so (include/octpt.h).

This is the Python-side view of the C ABI the Rust host would bind.  The
library is built in-tree by ``__graft_entry__.build()`` into ``octree_pathtracing_amd/lib``;
there is no fallback: importing a renderer without the library raises ``OctptLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_DIR = Path(__file__).resolve().parent / "lib"
LIB_PATH = LIB_DIR / "liboctpt.so"

OCTPT_ABI_VERSION = 4

OK = 0
ERR_INVALID_ARG = 1
ERR_OOM = 2
ERR_DEVICE = 3
NOT_READY = 4
ERR_UNSUPPORTED = 5
CANCELLED = 6
ERR_INTERNAL = 7

TEXTURE_COLOR = 0
TEXTURE_IMAGE = 1
RENDER_SHARD_COMPACT = 0x1
RENDER_MEGAKERNEL = 0x2
RENDER_KERNEL_TIMING = 0x4
RENDER_PREVIEW = 0x8
BUILD_COMPACT = 0x1  # OCTPT_BUILD_COMPACT
PRIM_NONE = 0xFFFFFFFF
PRIM_CUBOID_BIT = 0x80000000

STATUS_NAMES = {
    OK: "OK",
    ERR_INVALID_ARG: "INVALID_ARG",
    ERR_OOM: "OOM",
    ERR_DEVICE: "DEVICE_ERROR",
    NOT_READY: "NOT_READY",
    ERR_UNSUPPORTED: "UNSUPPORTED",
    CANCELLED: "CANCELLED",
    ERR_INTERNAL: "INTERNAL",
}


class OctptLibraryError(RuntimeError):
    """liboctpt.so is missing or failed to load (no CPU fallback exists)."""


class OctptError(RuntimeError):
    def __init__(self, status: int, message: str):
        self.status = status
        super().__init__(f"octpt error {STATUS_NAMES.get(status, status)}: {message}")


class Octant(C.Structure):
    _fields_ = [("child_mask", C.c_uint16), ("reserved", C.c_uint16), ("children", C.c_uint32 * 8)]


class Sphere(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("radius", C.c_float), ("material", C.c_uint32), ("reserved", C.c_uint32 * 3)]


class Cuboid(C.Structure):
    _fields_ = [("min", C.c_float * 3), ("max", C.c_float * 3), ("face_material", C.c_uint32 * 6)]


class Quad(C.Structure):
    """octpt_quad: Quad::new arguments (quad.rs:90-114), voxel-local."""
    _fields_ = [("origin", C.c_float * 3), ("material", C.c_uint32), ("u", C.c_float * 3), ("v", C.c_float * 3),
                ("texture_u_range", C.c_float * 2), ("texture_v_range", C.c_float * 2), ("reserved", C.c_uint32 * 2)]


class BlockModel(C.Structure):
    """octpt_block_model (gpu_structs/model.rs:14-21)."""
    _fields_ = [("flags", C.c_uint32), ("first_quad", C.c_uint32), ("quad_count", C.c_uint32),
                ("reserved", C.c_uint32)]


MODEL_NONE = 0xFFFFFFFF


class Block(C.Structure):
    """octpt_block: a block value's six face materials or its block model."""
    _fields_ = [("face_material", C.c_uint32 * 6), ("model", C.c_uint32), ("reserved", C.c_uint32)]
# numpy view of octpt_quad rows (Scene.quads)
QUAD_DTYPE = [("origin", "<f4", (3,)), ("material", "<u4"), ("u", "<f4", (3,)), ("v", "<f4", (3,)),
              ("texture_u_range", "<f4", (2,)), ("texture_v_range", "<f4", (2,)), ("reserved", "<u4", (2,))]


class Material(C.Structure):
    _fields_ = [
        ("ior", C.c_float), ("specular", C.c_float), ("emittance", C.c_float), ("roughness", C.c_float),
        ("metalness", C.c_float), ("texture_index", C.c_uint32), ("tint_index", C.c_uint32), ("flags", C.c_uint32),
    ]


class Texture(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("rgba", C.c_uint8 * 4), ("width", C.c_uint32), ("height", C.c_uint32),
                ("pixels", C.c_void_p)]


class Sun(C.Structure):
    _fields_ = [
        ("azimuth", C.c_float), ("altitude", C.c_float), ("radius", C.c_float), ("color", C.c_float * 4),
        ("apparent_color", C.c_float * 3), ("draw_texture", C.c_int32), ("texture_modification", C.c_int32),
        ("importance_sample_chance", C.c_float), ("importance_sample_radius", C.c_float), ("luminosity", C.c_float),
        ("texture_rgba", C.c_uint8 * 4), ("importance_sampling", C.c_int32), ("diffuse_sun", C.c_int32),
        ("sun_sampling", C.c_int32), ("strict_direct_light", C.c_int32), ("sun_luminosity", C.c_int32),
        ("luminosity_pdf", C.c_float),
    ]


class SceneDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_uint32), ("octants", C.c_void_p), ("octant_count", C.c_uint32), ("root", C.c_uint32),
        ("depth", C.c_uint32), ("leaf_first", C.c_void_p), ("leaf_count", C.c_void_p),
        ("leaf_table_size", C.c_uint32), ("leaf_prims", C.c_void_p), ("leaf_prim_count", C.c_uint32),
        ("spheres", C.c_void_p), ("sphere_count", C.c_uint32), ("cuboids", C.c_void_p), ("cuboid_count", C.c_uint32),
        ("materials", C.c_void_p), ("material_count", C.c_uint32), ("textures", C.c_void_p),
        ("texture_count", C.c_uint32), ("sun", Sun), ("emitters_enabled", C.c_int32), ("f_sub_surface", C.c_float),
        ("cuboid_model", C.c_void_p), ("models", C.c_void_p), ("model_count", C.c_uint32), ("quads", C.c_void_p),
        ("quad_count", C.c_uint32), ("blocks", C.c_void_p), ("block_count", C.c_uint32),
    ]


class ReferenceMaterial(C.Structure):
    """octpt_reference_material: textures::material::Material + its Texture (material.rs:91-101)."""
    _fields_ = [("index_of_refraction", C.c_float), ("specular", C.c_float), ("emittance", C.c_float),
                ("roughness", C.c_float), ("metalness", C.c_float), ("material_flags", C.c_uint32),
                ("tint_index", C.c_uint32), ("texture_kind", C.c_uint32), ("color", C.c_uint8 * 4),
                ("image_width", C.c_uint32), ("image_height", C.c_uint32), ("image_rgba", C.c_void_p)]


class ReferenceQuad(C.Structure):
    """octpt_reference_quad: geometry::quad::Quad field by field (quad.rs:7-17)."""
    _fields_ = [("origin", C.c_float * 3), ("u", C.c_float * 3), ("v", C.c_float * 3), ("w", C.c_float * 3),
                ("normal", C.c_float * 3), ("d", C.c_float), ("material_id", C.c_uint32),
                ("texture_u_range", C.c_float * 2), ("texture_v_range", C.c_float * 2)]


class ReferenceScene(C.Structure):
    """octpt_reference_scene: scene::Scene (scene/mod.rs:146-156) + the host's block table."""
    _fields_ = [("octants", C.c_void_p), ("octant_count", C.c_uint32), ("root", C.c_uint32), ("depth", C.c_uint32),
                ("blocks", C.c_void_p), ("block_count", C.c_uint32), ("models", C.c_void_p),
                ("model_count", C.c_uint32), ("quads", C.c_void_p), ("quad_count", C.c_uint32),
                ("materials", C.c_void_p), ("material_count", C.c_uint32), ("sun", Sun),
                ("emitters_enabled", C.c_int32), ("f_sub_surface", C.c_float)]


class Camera(C.Structure):
    _fields_ = [("eye", C.c_float * 3), ("direction", C.c_float * 3), ("up", C.c_float * 3), ("fov", C.c_float),
                ("aperture", C.c_float), ("focal_distance", C.c_float)]


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp_start", C.c_uint32), ("spp_count", C.c_uint32),
                ("max_depth", C.c_uint32), ("branch_count", C.c_uint32), ("seed", C.c_uint32),
                ("shard_index", C.c_uint32), ("shard_count", C.c_uint32), ("flags", C.c_uint32)]


# octpt_stats::drain order (OCTPT_STAT_*)
STAT_NAMES = ("paths", "segments", "esvo_steps", "sphere_tests", "cuboid_tests", "shade_events", "texel_reads",
              "block_tests", "issued_bytes")
STAT_COUNT = len(STAT_NAMES)


class Stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("segments", C.c_uint64), ("esvo_steps", C.c_uint64),
                ("sphere_tests", C.c_uint64), ("cuboid_tests", C.c_uint64), ("shade_events", C.c_uint64),
                ("texel_reads", C.c_uint64), ("launches", C.c_uint64), ("kernel_ms", C.c_double),
                ("extend_launches", C.c_uint64), ("shade_launches", C.c_uint64), ("extend_ms", C.c_double),
                ("shade_ms", C.c_double), ("build_ms", C.c_double), ("block_tests", C.c_uint64),
                ("issued_bytes", C.c_uint64), ("drain", C.c_uint64 * STAT_COUNT), ("pool_slots", C.c_uint64),
                ("chunk_items", C.c_uint64), ("wave_allocs", C.c_uint64), ("beam_restarts", C.c_uint64),
                ("hit_check_failures", C.c_uint64)]

    def as_dict(self) -> dict:
        d = {name: getattr(self, name) for name, _ in self._fields_}
        d["drain"] = dict(zip(STAT_NAMES, list(self.drain)))  # the drain kernel's share (in the totals)
        return d


class OctreeView(C.Structure):
    _fields_ = [("octants", C.c_void_p), ("octant_count", C.c_uint32), ("root", C.c_uint32), ("depth", C.c_uint32),
                ("leaf_first", C.c_void_p), ("leaf_count", C.c_void_p), ("leaf_table_size", C.c_uint32),
                ("leaf_prims", C.c_void_p), ("leaf_prim_count", C.c_uint32)]


# every symbol include/octpt.h declares, with its ctypes signature
_vp, _u32, _i32, _f = C.c_void_p, C.c_uint32, C.c_int32, C.c_float
SIGNATURES = {
    "octpt_abi_version": (_u32, []),
    "octpt_device_count": (_i32, []),
    "octpt_create": (_i32, [_i32, C.POINTER(_vp)]),
    "octpt_create_multi": (_i32, [_vp, _u32, C.POINTER(_vp)]),
    "octpt_device_entries": (_u32, [_vp]),
    "octpt_destroy": (None, [_vp]),
    "octpt_last_error": (C.c_char_p, [_vp]),
    "octpt_scene_upload": (_i32, [_vp, C.POINTER(SceneDesc)]),
    "octpt_scene_build_device": (_i32, [_vp, C.POINTER(SceneDesc), _u32]),
    "octpt_set_camera": (_i32, [_vp, C.POINTER(Camera)]),
    "octpt_get_camera": (_i32, [_vp, C.POINTER(Camera)]),
    "octpt_render": (_i32, [_vp, C.POINTER(RenderParams), _vp, _vp]),
    "octpt_render_device": (_i32, [_vp, C.POINTER(RenderParams), _vp, _vp, _vp]),
    "octpt_render_async": (_i32, [_vp, C.POINTER(RenderParams), _vp, _vp, C.POINTER(_vp)]),
    "octpt_frame_poll": (_i32, [_vp]),
    "octpt_frame_wait": (_i32, [_vp]),
    "octpt_frame_cancel": (_i32, [_vp]),
    "octpt_frame_release": (None, [_vp]),
    "octpt_tonemap_device": (_i32, [_vp, _vp, _vp, _u32, _vp]),
    "octpt_unshard_device": (_i32, [_vp, _u32, _u32, _u32, _vp, _u32, _vp, _vp]),
    "octpt_shard_pixels": (_u32, [_u32, _u32, _u32, _u32]),
    "octpt_set_tile_order": (_i32, [_vp, _u32, _u32, _vp]),
    "octpt_balance_tiles": (_i32, [_u32, _u32, _u32, _vp, _vp]),
    "octpt_intersect": (_i32, [_vp, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp]),
    "octpt_traversal_data": (_i32, [_vp, _u32, _u32, _u32, _vp, _f, _vp, _vp, _vp, _vp]),
    "octpt_get_stats": (_i32, [_vp, C.POINTER(Stats)]),
    "octpt_reset_stats": (_i32, [_vp]),
    "octpt_build_octree": (_i32, [_vp, _u32, _vp, _u32, _u32, C.POINTER(_vp)]),
    "octpt_build_octree_device": (_i32, [_vp, _vp, _u32, _vp, _u32, _u32, C.POINTER(_vp)]),
    "octpt_build_octree_ex": (_i32, [_vp, _u32, _vp, _u32, _u32, _u32, C.POINTER(_vp)]),
    "octpt_build_octree_device_ex": (_i32, [_vp, _vp, _u32, _vp, _u32, _u32, _u32, C.POINTER(_vp)]),
    "octpt_build_block_octree": (_i32, [_vp, _u32, _u32, _u32, C.POINTER(_vp)]),
    "octpt_scene_from_reference": (_i32, [C.POINTER(ReferenceScene), _vp, _vp, _vp, C.POINTER(SceneDesc)]),
    "octpt_octree_get_view": (_i32, [_vp, C.POINTER(OctreeView)]),
    "octpt_octree_free": (None, [_vp]),
}

_lib = None


def load(path: str | os.PathLike | None = None) -> C.CDLL:
    """Load liboctpt.so and bind every declared symbol; raises if missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # OCTPT_LIB: developer override to A/B differently built kernels (same ABI)
    p = Path(path) if path else Path(os.environ.get("OCTPT_LIB") or LIB_PATH)
    try:  # share torch's HIP runtime (same soname libamdhip64.so.7) when torch is present
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        pass
    if not p.exists():
        raise OctptLibraryError(f"{p} not built; run __graft_entry__.build() (no CPU fallback exists)")
    try:
        lib = C.CDLL(str(p))
    except OSError as e:  # pragma: no cover - depends on the box
        raise OctptLibraryError(f"cannot load {p}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.octpt_abi_version() != OCTPT_ABI_VERSION:
        raise OctptLibraryError("liboctpt ABI version mismatch")
    if path is None:
        _lib = lib
    return lib


def check(lib, ctx, status: int) -> None:
    if status != OK:
        msg = lib.octpt_last_error(ctx).decode() if ctx else ""
        raise OctptError(status, msg)
