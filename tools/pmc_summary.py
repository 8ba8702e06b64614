#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (counter_collection.csv) per kernel.

FETCH_SIZE and WRITE_SIZE are in KB.  gfx950 correction (MI355X_MICROARCH.md, HBM section):
FETCH_SIZE reports half the bytes of wide (16 B/lane) reads -> x2; WRITE_SIZE is exact.
  python tools/pmc_summary.py [--src=h16.hip] [--key=name=value ...] <fetch_dir> <write_dir> [kernel-name ...]
(the sha1 of the named csrc source is recorded, so a bench line only quotes counters measured on
the kernels it runs; --key records the workload the counters were taken on -- e.g. --key=n=50000000
--key=world=1 --key=mode=slab -- and a bench line quotes a record only when every key matches its
own run)
"""
import collections
import csv
import hashlib
import json
import os
import re
import sys


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] == counter:
            m = re.search(r"(\w+)(<[^(]*>)?\(", r["Kernel_Name"].replace("(anonymous namespace)", "anon"))
            name = m.group(1) if m else r["Kernel_Name"]
            vals[name].append(float(r["Counter_Value"]) * 1024.0)
    return vals


def main():
    args = sys.argv[1:]
    src_rel = "icp.hip"
    workload = {}
    while args and args[0].startswith("--"):
        a = args.pop(0)
        if a.startswith("--src="):  # the source whose kernels are summarised (sha1 recorded)
            src_rel = a[len("--src="):]
        elif a.startswith("--key="):  # the workload the counters were measured on
            k, v = a[len("--key="):].split("=", 1)
            workload[k] = int(v) if v.lstrip("-").isdigit() else v
    fdir, wdir = args[0], args[1]
    keys = args[2:] or ["k_icp_verify", "k_icp_octant", "k_icp_ring"]
    f, w = per_kernel(fdir, "FETCH_SIZE"), per_kernel(wdir, "WRITE_SIZE")
    out = {"source": f"{fdir}, {wdir}", "fetch_correction": 2.0, "kernels": {}}
    for k in keys:
        if k in f:
            fb = [2.0 * v for v in f[k]]
            wb = w.get(k, [])
            out["kernels"][k] = {"launches": len(fb), "fetch_bytes_avg": sum(fb) / len(fb),
                                 "write_bytes_avg": sum(wb) / len(wb) if wb else None}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "pointcloudprocess_amd", "csrc", src_rel)
    sha = hashlib.sha1(open(src, "rb").read()).hexdigest()
    if src_rel == "icp.hip":
        out["icp_hip_sha1"] = sha
    out["src"] = src_rel
    out["src_sha1"] = sha
    out["workload"] = workload
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
