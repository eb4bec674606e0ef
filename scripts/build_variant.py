"""Build a flag variant of liboctpt.so into build_variants/NAME/ (A/B experiments; select it on the
GPU box with OCTPT_LIB=build_variants/NAME/liboctpt.so).  Usage: build_variant.py NAME [-DFLAG ...]"""
import subprocess, sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import __graft_entry__ as g  # noqa: E402

name, extra = sys.argv[1], sys.argv[2:]
out = ROOT / "build_variants" / name / "liboctpt.so"
out.parent.mkdir(parents=True, exist_ok=True)
subprocess.run([g._hipcc(), *g.HIPCC_FLAGS, *extra, *map(str, g.SOURCES), "-o", str(out)], check=True)
print(out)
