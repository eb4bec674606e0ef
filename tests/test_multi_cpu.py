"""Multi-device contexts (octpt_create_multi) without a GPU: the tile bookkeeping that deals a
render's 8x8 tiles over the device entries and gathers them back (multi_slot, checked exhaustively against
the kernels' shard rule by tools/multi_layout_check.cpp), and the entry point's argument errors."""
import ctypes as C
import subprocess
from pathlib import Path

import pytest

from octree_pathtracing_amd import _lib

ROOT = Path(__file__).resolve().parents[1]


def test_multi_layout_bookkeeping(tmp_path):
    exe = tmp_path / "multi_layout_check"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    str(ROOT / "tools" / "multi_layout_check.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "mismatches 0" in out.stdout


def test_create_multi_arguments():
    lib = _lib.load()
    ctx = C.c_void_p()
    devs = (C.c_int32 * 2)(0, 0)
    assert lib.octpt_create_multi(devs, 2, None) == _lib.ERR_INVALID_ARG
    assert lib.octpt_create_multi(None, 2, C.byref(ctx)) == _lib.ERR_INVALID_ARG
    assert lib.octpt_create_multi(devs, 0, C.byref(ctx)) == _lib.ERR_INVALID_ARG
    assert lib.octpt_create_multi((C.c_int32 * 65)(), 65, C.byref(ctx)) == _lib.ERR_INVALID_ARG
    assert lib.octpt_device_entries(None) == 0
    if lib.octpt_device_count() > 0:
        pytest.skip("a GPU is visible: covered by tests/test_gpu_multi.py")
    assert lib.octpt_create_multi(devs, 2, C.byref(ctx)) == _lib.ERR_DEVICE and not ctx.value
