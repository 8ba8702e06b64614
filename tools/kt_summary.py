#!/usr/bin/env python3
"""Print the ICP kernels of rocprofv3 kernel_stats.csv files: python tools/kt_summary.py <dir>..."""
import csv, glob, os, sys
for d in sys.argv[1:]:
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if not f:
        continue
    print("==", d)
    for r in csv.DictReader(open(f[0])):
        n = r["Name"]
        if any(k in n for k in ("verify", "octant", "ring", "compact", "reduce_partials", "scan", "sort", "keys", "cell", "start")):
            print(f"  {n[:70]:70s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  tot {float(r['TotalDurationNs'])/1e6:8.2f} ms")
