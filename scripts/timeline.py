#!/usr/bin/env python3
"""Per-render timeline of a rocprofv3 kernel trace (…_kernel_trace.csv): renders are delimited by
wf_seed_kernel (beam_kernel, when present, precedes it).  For each render: wall time from its first kernel's
start to its last kernel's end, the time inside kernels by kind, the idle gaps between kernels (host launch /
steering latency), extend / shade launch counts and the tail (the time after the first extend shorter than
`tail_us`).  Usage: timeline.py TRACE_CSV [--skip N] [--tail-us 200]"""
import argparse
import csv
import json
import re
from collections import defaultdict


def kind_of(name: str) -> str:
    for k in ("beam_kernel", "wf_seed_kernel", "wf_extend_kernel", "wf_issued_extend_kernel", "wf_shade_kernel",
              "wf_drain_kernel", "wf_resolve_kernel", "multi_stage_kernel", "unshard_kernel", "tonemap_kernel"):
        if k in name:
            return k
    return re.sub(r"\(.*", "", name)[-40:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=0, help="renders to skip (warm-up)")
    ap.add_argument("--tail-us", type=float, default=200.0)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind_of(r["Kernel_Name"])))
    rows.sort()
    renders, cur = [], []
    for r in rows:
        if r[2] == "beam_kernel" or (r[2] == "wf_seed_kernel" and not (cur and cur[-1][2] == "beam_kernel")):
            if cur:
                renders.append(cur)
            cur = []
        cur.append(r)
    if cur:
        renders.append(cur)
    out = []
    for rend in renders[a.skip:]:
        t0, t1 = rend[0][0], max(e for _, e, _ in rend)
        busy = defaultdict(float)
        n = defaultdict(int)
        gaps, last_end = 0.0, rend[0][0]
        tail_start = None
        for s, e, k in rend:
            busy[k] += (e - s) / 1e3
            n[k] += 1
            gaps += max(0, s - last_end) / 1e3
            last_end = max(last_end, e)
            if k == "wf_extend_kernel" and tail_start is None and (e - s) / 1e3 < a.tail_us:
                tail_start = s
        out.append({"wall_us": round((t1 - t0) / 1e3, 1), "gaps_us": round(gaps, 1),
                    "tail_us": round((t1 - tail_start) / 1e3, 1) if tail_start else 0.0,
                    "busy_us": {k: round(v, 1) for k, v in sorted(busy.items())}, "launches": dict(n)})
    print(json.dumps({"renders": len(out), "per_render": out}, indent=1))


if __name__ == "__main__":
    main()
