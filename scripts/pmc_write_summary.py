"""Summarise scripts/gpu_pmc_write.sh: per (config, library, counter) the counter per wf_extend_kernel
launch (WRITE_SIZE in bytes, KiB x 1024) beside extend's algorithmic writes (8-B hit records: 8 B x
segments traced by extend per launch).  Usage: pmc_write_summary.py OUT_DIR  -> OUT_DIR/summary.json"""
import collections
import csv
import glob
import json
import os
import re
import sqlite3
import sys


def counter_per_kernel(d):
    tot, n = collections.defaultdict(float), collections.Counter()
    recs = []
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        recs += [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])) for r in csv.DictReader(open(f))]
    for f in glob.glob(d + "/**/*.db", recursive=True):  # rocpd output (the rocprofv3 default)
        with sqlite3.connect(f) as c:
            recs += list(c.execute("select kernel_name, counter_name, value from counters_collection"))
    for kname, cname, v in recs:
        m = re.search(r"(wf_\w+_kernel)", kname)
        if m:
            tot[(m.group(1), cname)] += v
            n[(m.group(1), cname)] += 1
    return tot, n


def main():
    out = sys.argv[1]
    rows = []
    for d in sorted(glob.glob(out + "/*_*_*")):
        if not os.path.isdir(d):
            continue
        cfg, lib, ctr = os.path.basename(d).split("_", 2)
        lines = [l for l in open(d + ".json") if l.startswith("{")]
        bench = json.loads(lines[-1])
        st = bench["stats_rank0"]
        segs = (st["segments"] - st["drain"]["segments"]) / st["extend_launches"]
        tot, n = counter_per_kernel(d)
        row = {"config": cfg, "lib": lib, "counter": ctr, "mrays_s": bench["value"],
               "extend_kernel_ms": bench["roofline"]["kernel_ms_avg"], "segments_per_launch": segs,
               "hit_record_bytes_per_launch": 8.0 * segs}
        for (k, c), v in tot.items():
            if c not in ctr.split("+"):
                continue
            per = v / n[(k, c)]
            if c in ("WRITE_SIZE", "FETCH_SIZE"):
                per *= 1024.0
            row[k if c == ctr else k + ":" + c] = per
        if "wf_extend_kernel" in row and ctr == "WRITE_SIZE":
            row["extend_write_over_hit_bytes"] = row["wf_extend_kernel"] / row["hit_record_bytes_per_launch"]
        rows.append(row)
        print(json.dumps(row))
    json.dump(rows, open(out + "/summary.json", "w"), indent=1)


if __name__ == "__main__":
    main()
