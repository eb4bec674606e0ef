"""The kernels' fixed-divisor integer division (octpt_internal.h udiv_magic / udiv_c: item -> tile -> pixel in the
seed, shade, resolve and beam kernels, round 6) against the C division: tools/udiv_check.cpp, built here with hipcc
(host code only) and run on the CPU.  A wrong quotient would move samples between pixels, which every render-parity
test would also catch on the GPU."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_udiv_matches_division(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists() and not shutil.which("hipcc"):
        pytest.skip("hipcc not available")
    exe = tmp_path / "udiv_check"
    subprocess.run([hipcc, "-O2", "-std=c++17", str(ROOT / "tools" / "udiv_check.cpp"), "-o", str(exe)], check=True,
                   capture_output=True, timeout=300)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "0 mismatches" in p.stdout
