import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

# The camera rays' beam start skips ESVO iterations over empty cells, so a render with
# it counts fewer ESVO iterations than the oracle, which restates the reference's walk from the cube
# entry.  The oracle-parity tests therefore run without it, which keeps the per-render ESVO iteration
# total an exact check of the traversal; tests/test_gpu_beam.py shows that renders with the beam equal
# those without it in everything else, bit for bit (and smoke() checks the shipped default against
# the oracle).
os.environ.setdefault("OCTPT_BEAM", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session", autouse=True)
def built_libraries():
    import __graft_entry__ as g

    g.build_library()
    g.build_oracle()
    return True
