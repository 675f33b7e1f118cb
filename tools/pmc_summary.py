"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh) per kernel and per launch.

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  The gfx950 x2 FETCH correction (MI355X_MICROARCH.md
"HBM") is calibrated for wide coalesced streaming reads; it is reported beside the raw value and
applied only where the kernel's reads are such streams (k_cg_update / k_xpby*).

    python tools/pmc_summary.py gpurun_out/<tag> [pmc_render_matvec.json]  > pmc_summary.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def _short(name):
    return name.replace("(anonymous namespace)", "anon").split("(")[0]


def load(pass_dir, counter):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                per[_short(row["Kernel_Name"])].append(float(row["Counter_Value"]))
    return per


def main(out_dir):
    fetch = load(os.path.join(out_dir, "pmc_fetch"), "FETCH_SIZE")
    write = load(os.path.join(out_dir, "pmc_write"), "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        fk = sum(f) / len(f) if f else 0.0
        wk = sum(w) / len(w) if w else 0.0
        res[k] = {"launches": max(len(f), len(w)), "fetch_bytes_per_launch_raw": fk * 1024,
                  "write_bytes_per_launch": wk * 1024, "fetch_bytes_per_launch_x2": 2 * fk * 1024}
    json.dump(res, sys.stdout, indent=1)
    print()
    # the dominant kernel's per-launch traffic, in the form bench.py reads (profiles/pmc_render_matvec.json)
    mv = [k for k in res if "k_render_matvec" in k]
    if mv and len(sys.argv) > 2:
        r = res[mv[0]]
        with open(sys.argv[2], "w") as f:
            json.dump({"kernel": mv[0], "P": 1000000, "width": 1920, "height": 1080,
                       "command": "rocprofv3 --pmc FETCH_SIZE | --pmc WRITE_SIZE (separate passes) -- "
                                  "python3 bench.py --no-cpu-baseline --steps 10 --warmup 3 --forward-steps 8 --no-side",
                       "round": os.environ.get("GSLM_PMC_ROUND", ""),
                       "fetch_bytes_per_launch_raw": r["fetch_bytes_per_launch_raw"],
                       "write_bytes_per_launch": r["write_bytes_per_launch"],
                       "hbm_bytes_per_launch": r["fetch_bytes_per_launch_x2"] + r["write_bytes_per_launch"],
                       "hbm_bytes_per_launch_raw": r["fetch_bytes_per_launch_raw"] + r["write_bytes_per_launch"],
                       "correction_note": "FETCH_SIZE / WRITE_SIZE are KiB per dispatch. FETCH_SIZE is doubled: "
                       "profiles/r02/pmc_calibration.json (tools/pmc_calib.hip, 1 GiB table) measures FETCH at "
                       "0.50 x the bytes of 16-B and 4-B coalesced streams and at 1.38 x the 48 B of a random "
                       "48-B record alone in its 128-B line (= half of the whole line the read pulls), so the "
                       "counter tallies memory-side 128-B line reads at 64 B for this kernel's record gathers "
                       "too; WRITE_SIZE is exact for 16-B coalesced stores and random 32-B rows (1.00)."},
                      f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
