"""Per-kernel timeline of the last full forward (k_preprocess .. k_render_fwd) in a rocprofv3 kernel trace:
    python tools/trace_forward.py <run_kernel_trace.csv>"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "k_render_fwd" in r["Kernel_Name"]]
i1 = ends[-1]
i0 = max(i for i in range(i1) if re.search(r"k_preprocess(_dma)?<", rows[i]["Kernel_Name"]))
t0 = int(rows[i0]["Start_Timestamp"])
prev = None
busy = 0
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{name[:44]:44s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  at {(s - t0) / 1e3:8.1f}")
    prev = e
print(f"forward span {(prev - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
