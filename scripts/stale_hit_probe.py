"""The round-3 stale-hit defect: block_leaf_test with its hit fields written after the alpha
test's divergent branch (build_variants/prefix: the pre-fix order on today's sources; prefix_check: the same
with -DOCTPT_CHECK_HITS) against the product library, on the alpha-face world of tests/test_gpu_blocks.py.
Round 5: variant slotleak_check (-DOCTPT_SLOT_LEAK_PROBE -DOCTPT_CHECK_HITS: advancing lanes take the node slot
they never loaded) is the negative control of the check build's slot poisoning (SLOT_CHECK).
Prints one JSON line: per-variant pixels differing from the product render (3 renders each) and the check
build's hit_check_failures.  Usage: stale_hit_probe.py [VARIANT ...] (default: prefix prefix_check)"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    import torch

    from octree_pathtracing_amd.renderer import HipRenderer
    from tests.test_gpu_blocks import _alpha_world
    from tests.test_gpu_parity import gpu_render

    sc, cam, rs = _alpha_world()
    out = {"scene": "tests/test_gpu_blocks.py::_alpha_world", "size": [rs.width, rs.height, rs.spp]}
    prod = HipRenderer(device=0)
    ref = gpu_render(torch, prod, sc, cam, rs)
    prod.close()
    for name in sys.argv[1:] or ("prefix", "prefix_check"):
        lib = ROOT / "build_variants" / name / "liboctpt.so"
        r = HipRenderer(device=0, lib_path=str(lib))
        runs = []
        for _ in range(3):
            a = gpu_render(torch, r, sc, cam, rs)
            diff = int((a[0].view(np.uint32) != ref[0].view(np.uint32)).any(-1).sum())
            runs.append({"pixels_differing": diff, "hit_check_failures": a[2]["hit_check_failures"]})
        r.close()
        out[name] = runs
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
