#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the LM tile kernels per library build (tools/mv_ab.py, separate --pmc passes):
#   bash tools/pmc_ab.sh <tag> <build_dir>...      (gpurun, from the repo root)
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
ROOT=$(pwd)
for L in "$@"; do
  OUT=$ROOT/gpurun_out/$TAG/$L; mkdir -p $OUT
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && GSLM_ABI_ANY=1 GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -s KILL 180 rocprofv3 --pmc $c \
       -f csv -d $OUT/$c -o run -- python3 $ROOT/tools/mv_ab.py $L --reps 3 --out /tmp/gslm_ab > /dev/null 2> $OUT/$c.err) || exit 1
  done
  echo "== $L"
  python3 - $OUT <<'PY'
import csv, glob, sys
out = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = {}
    for p in glob.glob(f"{out}/{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gslm::", "")
            if any(x in k for x in ("k_render_matvec", "k_render_fwd", "k_render_jv", "k_gather_lm", "k_render_bwd")):
                acc.setdefault(k, []).append(float(r["Counter_Value"]) * 1024)
    for k, v in sorted(acc.items()):
        scale = 2 if c == "FETCH_SIZE" else 1  # calibrated: FETCH tallies 128-B line reads at 64 B
        print(f"  {c:10s} {k:34s} {scale * sum(v) / len(v) / 1e6:9.1f} MB per launch (n={len(v)})")
PY
done
