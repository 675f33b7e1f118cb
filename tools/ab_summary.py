"""Summarise an ab_run.sh directory: per build, the median of each *_ms field over its runs.
    python tools/ab_summary.py gpurun_out/<tag>"""
import glob
import json
import os
import statistics
import sys

runs = {}
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    name = os.path.basename(f)[:-5]
    tag = name.split(".", 1)[1] if "." in name else name
    try:
        d = json.load(open(f))
    except ValueError:
        continue
    runs.setdefault(tag, []).append(d)
keys = sorted({k for ds in runs.values() for d in ds for k in d if k.endswith("_ms")})
print("build".ljust(16) + "".join(k.replace("_ms", "").rjust(22) for k in keys))
for tag, ds in runs.items():
    row = []
    for k in keys:
        vals = [d[k] for d in ds if isinstance(d.get(k), (int, float))]
        row.append(f"{statistics.median(vals):.4f} ({len(vals)})" if vals else "-")
    print(tag.ljust(16) + "".join(r.rjust(22) for r in row))
