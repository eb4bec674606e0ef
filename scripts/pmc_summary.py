"""Summarise rocprofv3 counter CSVs per kernel: python scripts/pmc_summary.py DIR..."""
import collections, csv, sys, glob
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            import re; m = re.search(r"(\w+_kernel|\w+Functor\w*|__amd\w+)", r["Kernel_Name"]); k = m.group(1) if m else r["Kernel_Name"][:40]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            agg[k]["_vgpr"] = float(r["VGPR_Count"])
        print("==", f)
        for k, c in agg.items():
            print(" ", k, {n: f"{v:.4g}" for n, v in sorted(c.items())})
    for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
        print("==", f)
        for r in csv.DictReader(open(f)):
            import re; m = re.search(r'(\w+_kernel|__amd\w+|\w+Functor)', r['Name']); print(f"  {(m.group(1) if m else r['Name'][:40]):42s} calls {r['Calls']:>6s} total {float(r['TotalDurationNs'])/1e6:9.2f} ms  avg {float(r['AverageNs'])/1e3:9.1f} us  {float(r['Percentage']):5.1f}%")
