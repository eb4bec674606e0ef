"""L2-to-fabric traffic per launch of the wavefront kernels from rocprofv3 --pmc FETCH_SIZE /
WRITE_SIZE passes (separate passes: the two do not fit one TCC pass).

Corrections per MI355X_MICROARCH.md (HBM section): FETCH_SIZE / WRITE_SIZE are in KiB and count
L2 memory-side requests (Infinity-Cache hits included, so this upper-bounds HBM bytes); on gfx950
FETCH_SIZE reports 1/2 of the bytes of wide reads, so it is doubled.
The FETCH_SIZE factor defaults to that halving (2); FACTOR overrides it with a calibrated value
(tools/fetch_calib.hip, profiles/fetch_calib.json) and NOTE says where it came from.
With TCC_DIR (a --pmc TCC_HIT_sum TCC_MISS_sum pass) the L2 hit rate per kernel is recorded too.
SOURCE (default: the one-step bench) names the profiled command.
Usage: python scripts/pmc_traffic.py FETCH_DIR WRITE_DIR CONFIG OUT_JSON [FACTOR NOTE [TCC_DIR [SOURCE]]]"""
import collections
import csv
import glob
import json
import re
import sys

KERNELS = ("wf_extend_kernel", "wf_shade_kernel", "wf_seed_kernel", "wf_resolve_kernel")


def per_kernel(d, counter):
    tot, n = collections.Counter(), collections.Counter()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            m = re.search(r"(wf_\w+_kernel)", r["Kernel_Name"])
            if not m:
                continue
            tot[m.group(1)] += float(r["Counter_Value"])
            n[m.group(1)] += 1
    return tot, n


def main():
    fetch_dir, write_dir, config, out = sys.argv[1:5]
    factor = float(sys.argv[5]) if len(sys.argv) > 5 else 2.0
    note = sys.argv[6] if len(sys.argv) > 6 else "gfx950 FETCH_SIZE halving of 16-B streaming reads"
    tcc_dir = sys.argv[7] if len(sys.argv) > 7 and sys.argv[7] else None
    source = sys.argv[8] if len(sys.argv) > 8 else "python3 bench.py --steps 1"
    ft, fn = per_kernel(fetch_dir, "FETCH_SIZE")
    wt, wn = per_kernel(write_dir, "WRITE_SIZE")
    res = {"config": config, "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, {source}",
           "fetch_factor": factor,
           "correction": f"bytes = {factor} * FETCH_SIZE[KiB] * 1024 + WRITE_SIZE[KiB] * 1024 ({note})",
           "raw": {}}
    for k in KERNELS:
        if fn[k] == 0 or wn[k] == 0:
            continue
        fetch = factor * ft[k] * 1024.0 / fn[k]
        res["raw"][k] = {"fetch_size_kib_per_launch": ft[k] / fn[k], "write_size_kib_per_launch": wt[k] / wn[k]}
        write = wt[k] * 1024.0 / wn[k]
        res[k] = {"launches": fn[k], "fetch_bytes_per_launch": int(fetch), "write_bytes_per_launch": int(write),
                  "bytes_per_launch": int(fetch + write)}
    if tcc_dir:
        ht, _ = per_kernel(tcc_dir, "TCC_HIT_sum")
        mt, _ = per_kernel(tcc_dir, "TCC_MISS_sum")
        for k in KERNELS:
            if k in res and ht[k] + mt[k] > 0:
                res[k]["l2_hit_rate"] = round(ht[k] / (ht[k] + mt[k]), 4)
    open(out, "w").write(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
