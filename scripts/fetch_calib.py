"""FETCH_SIZE calibration (tools/fetch_calib.hip): per access shape, the ratio of the footprint the
tool printed to rocprofv3's FETCH_SIZE bytes.  Usage:
    python scripts/fetch_calib.py TOOL_STDOUT PMC_DIR OUT_JSON
FETCH_SIZE is in KiB (MI355X_MICROARCH.md, HBM).  Dispatches are taken in launch order, skipping the
runtime's own fill/copy kernels: stream16, gather<uint2>, gather<uint4>, gather<uint2> (warm-up of
the resident table), gather<uint2> (16 passes over it)."""
import csv
import glob
import json
import sys


def main():
    tool_out, pmc_dir, out = sys.argv[1:4]
    known = {}
    for line in open(tool_out):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            known[d["kernel"]] = d
    rows = []
    for f in glob.glob(pmc_dir + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == "FETCH_SIZE" and "rocclr" not in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    rows.sort()
    names = ["stream16", "gather8", "gather16", "warm", "gather8_l3"]
    if len(rows) != len(names):
        raise SystemExit(f"expected {len(names)} dispatches, found {len(rows)}: {rows}")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE -- tools/fetch_calib (MI355X)"}
    for name, (_, kname, fetch) in zip(names, rows):
        if name == "warm":
            continue
        k = known[name]
        e = {"kernel": kname, "fetch_size_bytes": int(fetch)}
        if name == "stream16":
            e["footprint_bytes"] = k["footprint_bytes"]
            e["footprint_over_fetch"] = round(k["footprint_bytes"] / fetch, 4)
        elif name in ("gather8", "gather16"):
            e.update({"reads": k["reads"], "lines64": k["lines64"], "lines128": k["lines128"]})
            e["lines64_bytes_over_fetch"] = round(k["lines64"] * 64 / fetch, 4)
            e["lines128_bytes_over_fetch"] = round(k["lines128"] * 128 / fetch, 4)
            e["fetch_bytes_per_read"] = round(fetch / k["reads"], 2)
        else:
            e.update({"reads": k["reads"], "table_bytes": k["table_bytes"]})
            e["fetch_bytes_per_read"] = round(fetch / k["reads"], 3)
        res[name] = e
    open(out, "w").write(json.dumps(res, indent=1) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
