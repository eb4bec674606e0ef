#!/usr/bin/env python3
"""ESVO iteration-class statistics from the oracle (diagnostic; test infrastructure only).

Builds oracle/cpu_ref.c with -DREF_ESVO_TRACE into /tmp, renders a config at a reduced size on one
thread and classifies every reference iteration (octree_traversal.rs:127-300): advance over an
absent child, leaf test (miss / hit), descend, advance past a present child not entered, and pops.
It then counts how many kernel iterations a step that folds runs of absent-child advances into the
preceding iteration would take (sibling skipping).

usage: tools/esvo_trace.py CONFIG [W H SPP]
"""
import ctypes as C
import subprocess
import sys
from collections import Counter
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C3"
    from octree_pathtracing_amd import scene as S
    from oracle import cpu_ref

    lib = Path("/tmp/libcpu_ref_trace.so")
    subprocess.run(["gcc", "-O2", "-std=c11", "-D_GNU_SOURCE", "-fPIC", "-ffp-contract=off", "-DREF_ESVO_TRACE",
                    "-shared", "-o", str(lib), str(ROOT / "oracle" / "cpu_ref.c"), "-lm", "-pthread"], check=True)
    L = cpu_ref.load(lib)
    sc, cam, rs = S.make_config(cfg)
    W, H, spp = (int(a) for a in sys.argv[2:5]) if len(sys.argv) > 4 else (192, 108, 2)
    cap = 400_000_000
    buf = np.zeros(cap, np.uint8)
    L.ref_esvo_trace_set.argtypes = [C.c_void_p, C.c_size_t]
    L.ref_esvo_trace_len.restype = C.c_size_t
    L.ref_esvo_trace_set(buf.ctypes.data, cap)
    _, _, st = cpu_ref.render(sc, cam, W, H, spp, max_depth=rs.max_depth, seed=rs.seed, threads=1, forward=True)
    n = L.ref_esvo_trace_len()
    t = buf[:n]
    kind = t & 7
    pop = (t & 8) != 0
    first = (t & 16) != 0
    bounce = (t & 32) != 0
    print(f"{cfg} {W}x{H}x{spp}: {st['segments']} segments, {n} iterations ({n / st['segments']:.1f}/segment)")
    names = {0: "absent-advance", 1: "leaf miss", 2: "leaf hit", 3: "descend", 4: "present, not entered"}
    for k, v in sorted(Counter(kind.tolist()).items()):
        print(f"  {names[k]:22s} {v / n:6.1%}   popped {np.mean(pop[kind == k]):.1%}")
    # the leading descends of each ray (iterations before its first non-descend): what a start at the
    # ray's origin cell would skip (bounce rays from their leaf)
    ray_id = np.cumsum(first) - 1
    nd = kind != 3
    first_nd = np.full(ray_id[-1] + 1, n, np.int64)
    np.minimum.at(first_nd, ray_id[nd], np.nonzero(nd)[0])
    starts = np.nonzero(first)[0]
    lead = np.minimum(first_nd, np.append(starts[1:], n)) - starts
    rb = bounce[starts]
    print(f"  leading descends: bounce rays {lead[rb].mean():.2f} per ray ({rb.mean():.1%} of rays), camera rays "
          f"{lead[~rb].mean():.2f}; bounce rays' leading descends = {lead[rb].sum() / n:.1%} of all iterations, "
          f"{lead[rb].sum() / max(int((bounce).sum()), 1):.1%} of bounce rays' iterations")
    # folding: an absent-advance folds into the previous iteration of the same ray when that
    # iteration did not pop (K: at most K folds per iteration); optionally after a pop too
    seq = kind.tolist()
    pops = pop.tolist()
    firsts = first.tolist()
    for after_pop in (False, True):
        for K in (1, 2, 3, 8):
            kept = 0
            chain = 0
            prev_pop = True
            for i in range(n):
                fold = (seq[i] == 0 and not firsts[i] and chain < K and (after_pop or not prev_pop))
                if fold:
                    chain += 1
                else:
                    kept += 1
                    chain = 0
                prev_pop = pops[i] if not fold else (prev_pop or pops[i]) if False else pops[i]
            print(f"  fold K={K} after_pop={after_pop}: {kept / n:.3f} of iterations remain")


if __name__ == "__main__":
    main()
