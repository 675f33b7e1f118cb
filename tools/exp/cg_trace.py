"""Experiment helper: the CG loop's iterations in a rocprofv3 kernel trace -- start-to-start time between
consecutive k_render_matvec launches, and the kernels (duration, gap before) of one median iteration.
    python tools/exp/cg_trace.py <run_kernel_trace.csv> [label]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_render_matvec<false>" in r["Kernel_Name"]]
starts = [int(rows[i]["Start_Timestamp"]) for i in idx]
# iterations: consecutive matvecs less than 2 ms apart, in runs of at least 8
its = []
run = [0]
for k in range(1, len(idx)):
    if starts[k] - starts[k - 1] < 2_000_000:
        run.append(k)
    else:
        if len(run) >= 8:
            its.append(run)
        run = [k]
if len(run) >= 8:
    its.append(run)
label = sys.argv[2] if len(sys.argv) > 2 else ""
for run in its:
    d = sorted((starts[run[j + 1]] - starts[run[j]]) / 1e3 for j in range(len(run) - 1))
    print(f"{label} run of {len(run)} matvecs: start-to-start us median {d[len(d) // 2]:.1f} min {d[0]:.1f} max {d[-1]:.1f}")
    # the iteration at the median
    dd = [(starts[run[j + 1]] - starts[run[j]], j) for j in range(len(run) - 1)]
    dd.sort()
    j = dd[len(dd) // 2][1]
    a, b = idx[run[j]], idx[run[j + 1]]
    prev = None
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        print(f"   {name[:48]:48s} {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}")
        prev = e
