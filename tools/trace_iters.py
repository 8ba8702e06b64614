#!/usr/bin/env python3
"""Per-iteration durations of the ICP passes of the LAST registration in a rocprofv3 kernel
trace, plus the pre-iteration (build + sort) span:  python tools/trace_iters.py <trace_dir>"""
import csv, glob, os, sys
f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
d = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
sel = lambda k: [r for r in rows if k in r["Kernel_Name"]]
oc, ve, ri, t1 = sel("k_icp_octant"), sel("k_icp_verify"), sel("k_icp_ring"), sel("k_icp_tier1")
n = 20
print("octant", [round(d(r)) for r in oc[-n:]], round(sum(d(r) for r in oc[-n:])))
print("tier1 ", [round(d(r)) for r in t1[-(n - 1):]], round(sum(d(r) for r in t1[-(n - 1):])))
print("verify", [round(d(r)) for r in ve[-(n - 1):]], round(sum(d(r) for r in ve[-(n - 1):])))
print("ring  ", [round(d(r)) for r in ri[-n:]], round(sum(d(r) for r in ri[-n:])))
start, end = int(oc[-n]["Start_Timestamp"]), int(ri[-1]["End_Timestamp"])
prev = int(ri[-n - 1]["End_Timestamp"]) if len(ri) > n else int(rows[0]["Start_Timestamp"])
print(f"iterations span {(end - start) / 1e3:.0f} us, pre-iteration span {(start - prev) / 1e3:.0f} us")
# everything else inside the iterations span, by kernel
other = {}
for r in rows:
    if start <= int(r["Start_Timestamp"]) <= end and not any(k in r["Kernel_Name"] for k in
                                                               ("k_icp_octant", "k_icp_verify", "k_icp_ring", "k_icp_tier1")):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
        other[k] = other.get(k, 0.0) + d(r)
for k, v in sorted(other.items(), key=lambda kv: -kv[1])[:12]:
    print(f"  other {v:9.0f} us  {k}")
# the pre-iteration span (index build + query sort) of that registration, by kernel
pre = {}
for r in rows:
    if prev <= int(r["Start_Timestamp"]) < start:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:70]
        pre[k] = pre.get(k, 0.0) + d(r)
for k, v in sorted(pre.items(), key=lambda kv: -kv[1])[:16]:
    print(f"  pre   {v:9.0f} us  {k}")
