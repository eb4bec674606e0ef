"""The C-ABI boundary without a GPU: liboctpt.so loads, exports exactly what include/octpt.h
declares, the ctypes mirrors match the C layouts (gcc probe), and device-free entry points
(version, device count, octree builder, argument validation) behave."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

from octree_pathtracing_amd import _lib

ROOT = Path(__file__).resolve().parents[1]
HEADER = ROOT / "include" / "octpt.h"

# C struct name -> ctypes mirror in _lib
STRUCTS = {"octpt_octant": "Octant", "octpt_sphere": "Sphere", "octpt_cuboid": "Cuboid",
           "octpt_material": "Material", "octpt_texture": "Texture", "octpt_sun": "Sun",
           "octpt_scene_desc": "SceneDesc", "octpt_camera": "Camera", "octpt_render_params": "RenderParams",
           "octpt_stats": "Stats", "octpt_octree_view": "OctreeView", "octpt_quad": "Quad",
           "octpt_block_model": "BlockModel", "octpt_block": "Block",
           "octpt_reference_material": "ReferenceMaterial", "octpt_reference_quad": "ReferenceQuad",
           "octpt_reference_scene": "ReferenceScene"}


def header_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    names = set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(octpt_\w+)\s*\(", text, flags=re.M))
    return names


def exported_symbols(path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(path)], check=True, capture_output=True, text=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


@pytest.fixture(scope="module")
def lib():
    return _lib.load()


def test_header_and_exports_agree(lib):
    declared = header_functions()
    assert len(declared) >= 20
    exported = {s for s in exported_symbols(_lib.LIB_PATH) if s.startswith("octpt_")}
    assert declared == exported, (declared ^ exported)
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    for name in declared:
        assert hasattr(lib, name)


def test_struct_layouts_match_gcc(tmp_path):
    probe = tmp_path / "probe.c"
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void) {"]
    for c_name in STRUCTS:
        lines.append(f'    printf("{c_name} %zu %zu\\n", sizeof({c_name}), _Alignof({c_name}));')
    lines.append("    return 0;\n}")
    probe.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", str(probe), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    for line in out.splitlines():
        name, size, align = line.split()
        mirror = getattr(_lib, STRUCTS[name])
        assert C.sizeof(mirror) == int(size), (name, C.sizeof(mirror), size)
        assert C.alignment(mirror) <= int(align)


def test_reference_layout_sizes():
    """Octant is 36 B like new_octree::Octant (new_octree.rs:852-858 prints size_of::<Octant>())
    and the material record is GPUMaterial's 32 B (gpu_material.rs:7-18)."""
    assert C.sizeof(_lib.Octant) == 36
    assert C.sizeof(_lib.Material) == 32


def test_version_and_devices(lib):
    assert lib.octpt_abi_version() == _lib.OCTPT_ABI_VERSION == 4
    assert lib.octpt_device_count() >= 0


def test_create_without_device(lib):
    if lib.octpt_device_count() > 0:
        pytest.skip("a GPU is visible: covered by the gpu tests")
    ctx = C.c_void_p()
    st = lib.octpt_create(0, C.byref(ctx))
    assert st == _lib.ERR_DEVICE and not ctx.value
    assert lib.octpt_create(0, None) == _lib.ERR_INVALID_ARG


def test_null_context_calls_fail_cleanly(lib):
    assert lib.octpt_scene_upload(None, None) == _lib.ERR_INVALID_ARG
    assert lib.octpt_scene_build_device(None, None, 0) == _lib.ERR_INVALID_ARG
    assert lib.octpt_set_camera(None, None) == _lib.ERR_INVALID_ARG
    assert lib.octpt_render(None, None, None, None) == _lib.ERR_INVALID_ARG
    assert lib.octpt_get_stats(None, None) == _lib.ERR_INVALID_ARG
    assert lib.octpt_frame_poll(None) == _lib.ERR_INVALID_ARG
    lib.octpt_destroy(None)  # no-op
    lib.octpt_frame_release(None)
    assert lib.octpt_last_error(None)  # never NULL


def test_builder_argument_errors(lib):
    out = C.c_void_p()
    assert lib.octpt_build_octree(None, 0, None, 0, 0, C.byref(out)) == _lib.ERR_INVALID_ARG  # depth 0
    assert lib.octpt_build_octree(None, 0, None, 0, 22, C.byref(out)) == _lib.ERR_INVALID_ARG  # > kMaxDepth
    assert lib.octpt_build_octree(None, 5, None, 0, 4, C.byref(out)) == _lib.ERR_INVALID_ARG  # NULL spheres
    assert lib.octpt_build_octree(None, 0, None, 0, 4, None) == _lib.ERR_INVALID_ARG


def test_shard_pixels_partition(lib):
    for W, H, N in [(1920, 1080, 8), (70, 45, 3), (1, 1, 4), (9, 17, 2)]:
        counts = [lib.octpt_shard_pixels(W, H, k, N) for k in range(N)]
        tiles = ((W + 7) // 8) * ((H + 7) // 8)
        assert sum(counts) == sum(64 * len(range(k, tiles, N)) for k in range(N))
        assert max(counts) - min(counts) <= 64


def test_device_build_descriptor():
    """octpt_scene_build_device's descriptor (Scene.to_desc(octree=False)): octree fields NULL / 0,
    the build depth set, primitives and tables as for octpt_scene_upload."""
    from octree_pathtracing_amd import scene as S

    sc, _, _ = S.make_config("tiny", build=False)
    d, keep = sc.to_desc(octree=False, depth=7)
    assert not d.octants and d.octant_count == 0 and d.root == 0 and d.depth == 7
    assert not d.leaf_first and not d.leaf_count and d.leaf_table_size == 0
    assert not d.leaf_prims and d.leaf_prim_count == 0
    assert d.sphere_count == len(sc.spheres) and d.cuboid_count == len(sc.cuboids)
    assert d.material_count == len(sc.materials) and d.texture_count == len(sc.textures)
    sc.build_octree(5)
    d2, keep2 = sc.to_desc()
    assert d2.octants and d2.octant_count == sc.octree.octant_count and d2.depth == 5
