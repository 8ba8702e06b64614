#!/usr/bin/env python3
"""One line per bench JSON line of the A/B files in a gpurun output dir:
  python tools/ab_summary.py gpurun_out/<tag>"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(os.path.join(sys.argv[1], "c*_ab_*.jsonl"))):
    for line in open(f):
        line = line.strip()
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        r = d.get("roofline") or {}
        pr = (d.get("per_rank") or [{}])[0]
        print(f"{os.path.basename(f):24s} {d['value']:10.2f} {d['unit'][:12]:12s} {d['ms_per_step']:8.2f} ms/step  "
              f"kernel {r.get('kernel_avg_ms')} ms  frac {r.get('frac')}  pre {pr.get('pre_iteration_ms')}")
