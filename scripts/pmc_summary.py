"""Summarise rocprofv3 outputs under a directory: kernel stats + per-kernel, per-dispatch counter means."""
import csv, glob, os, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
kfilter = sys.argv[2] if len(sys.argv) > 2 else "add_"
for f in sorted(glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f}")
agg = {}
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        if kfilter not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0][-40:]
        agg.setdefault(k, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
for k, d in agg.items():
    print("--", k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
