#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the box (tools/pmc_calib.hip, built here beforehand):
#   hipcc --offload-arch=gfx950 -O3 tools/pmc_calib.hip -o tools/pmc_calib
#   gpurun -- 'bash tools/pmc_calib.sh'
# Separate --pmc passes; prints reported / known bytes per kernel (averages over the 3 launches each).
set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmc_calib
mkdir -p $OUT
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/fetch -o run -- $ROOT/tools/pmc_calib > $OUT/known.json 2> $OUT/fetch.err) \
&& (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/write -o run -- $ROOT/tools/pmc_calib > /dev/null 2> $OUT/write.err) \
&& python3 - "$OUT" <<'PY'
import csv, glob, json, sys
out = sys.argv[1]
known = json.loads(open(f"{out}/known.json").read().strip().splitlines()[-1])["known_bytes"]
def load(sub, counter):
    acc = {}
    for p in glob.glob(f"{out}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] != counter:
                continue
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc.setdefault(k, []).append(float(r["Counter_Value"]) * 1024)  # KiB per dispatch
    return {k: sum(v) / len(v) for k, v in acc.items()}
f, w = load("fetch", "FETCH_SIZE"), load("write", "WRITE_SIZE")
res = {}
for k, kb in known.items():
    res[k] = {"known_bytes": kb, "fetch_bytes": f.get(k), "write_bytes": w.get(k),
              "fetch_over_known": f.get(k, 0) / kb, "write_over_known": w.get(k, 0) / kb}
json.dump(res, open(f"{out}/calib.json", "w"), indent=1)
for k, r in res.items():
    print(f"{k:12s} known {r['known_bytes'] / 1e6:9.1f} MB  FETCH/known {r['fetch_over_known']:.3f}  WRITE/known {r['write_over_known']:.3f}")
PY
