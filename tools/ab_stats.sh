#!/bin/bash
# A/B kernel stats of two library builds: bash tools/ab_stats.sh <tag> <build_dir_a> <build_dir_b>
TAG=$1; shift
export TMPDIR=/tmp
ROOT=$(pwd)
for L in "$@"; do
  OUT=gpurun_out/$TAG/$L
  mkdir -p "$OUT"
  (cd /tmp && GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv \
     -d "$ROOT/$OUT/stats" -o run -- python3 "$ROOT/bench.py" --no-cpu-baseline --steps 10 --warmup 3 --forward-steps 8 \
     > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/err.log") || exit 1
done
python3 - "$TAG" "$@" <<'PY'
import csv, sys
tag, libs = sys.argv[1], sys.argv[2:]
tabs = []
for L in libs:
    rows = list(csv.DictReader(open(f"gpurun_out/{tag}/{L}/stats/run_kernel_stats.csv")))
    tabs.append({r["Name"].replace("(anonymous namespace)", "anon").split("(")[0][:58]: (int(r["Calls"]), float(r["AverageNs"]) / 1e3) for r in rows})
names = sorted(tabs[0], key=lambda k: -tabs[0][k][0] * tabs[0][k][1])[:24]
print(f"{'kernel':58s} " + " ".join(f"{L:>14s}" for L in libs))
for n in names:
    print(f"{n:58s} " + " ".join(f"{t.get(n, (0, 0))[1]:11.1f} us" for t in tabs))
PY
