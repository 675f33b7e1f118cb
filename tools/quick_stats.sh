#!/bin/bash
# Kernel-trace stats of a short bench run: gpurun_out/<tag>/stats/run_kernel_stats.csv + a digest.
TAG=${1:-qs}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/stats" -o run \
   -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 3 --forward-steps 8 > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/err.log") \
&& python3 - "$OUT" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/stats/run_kernel_stats.csv")))
for r in rows[:22]:
    name = r["Name"].replace("(anonymous namespace)", "anon").split("(")[0][:60]
    print(f"{name:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.1f} us")
PY
