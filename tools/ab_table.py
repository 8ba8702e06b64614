"""Summarise gpurun_out/<tag>/all.jsonl: per label, ms per registration and per-iteration kernel ms."""
import collections, json, sys

runs = collections.defaultdict(list)
for line in open(sys.argv[1]):
    d = json.loads(line)
    runs[d["label"]].append((d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d["value"]))
for k, v in runs.items():
    ms = [x[0] for x in v]
    it = [x[1] for x in v]
    print(f"{k:12s} ms/step {' '.join(f'{m:7.3f}' for m in ms)}  mean {sum(ms)/len(ms):7.3f}  "
          f"iter-kernel {sum(it)/len(it):6.4f}  non-iter {sum(ms)/len(ms) - 20 * sum(it)/len(it):6.3f}")
