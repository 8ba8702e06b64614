#!/usr/bin/env python3
"""Average each PMC counter per kernel over the passes written by tools/pmc_passes.sh.
  python tools/pmc_table.py <outdir> [kernel-substring ...]"""
import collections
import csv
import glob
import os
import re
import sys

out = sys.argv[1]
keys = sys.argv[2:] or ["k_icp_octant"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(out, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+)(<[^(]*>)?\(", r["Kernel_Name"].replace("(anonymous namespace)", "anon"))
        name = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"]
        if any(k in name for k in keys):
            vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"  {c:40s} {sum(v) / len(v):16.4g}   (n={len(v)})")
