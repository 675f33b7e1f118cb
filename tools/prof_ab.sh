#!/bin/bash
# rocprofv3 kernel stats of tools/mv_ab.py for library builds: bash tools/prof_ab.sh <tag> <build_dir>...
# (extra mv_ab arguments in MVAB_ARGS); prints each build's per-kernel average for the main LM kernels.
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
ROOT=$(pwd)
for L in "$@"; do
  OUT=gpurun_out/$TAG/$L
  mkdir -p $OUT
  (cd /tmp && GSLM_ABI_ANY=1 GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 rocprofv3 --kernel-trace \
     --stats -f csv -d $ROOT/$OUT -o run -- python3 $ROOT/tools/mv_ab.py $L --reps 5 --out /tmp/gslm_ab $MVAB_ARGS \
     > $ROOT/$OUT/ab.json 2> $ROOT/$OUT/err.log) || exit 1
  echo "== $L"
  python3 - "$(find $OUT -name '*kernel_stats.csv' | head -1)" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(k in n for k in ("k_gather_lm", "k_render_matvec", "k_preprocess_jvp", "k_cg_update", "k_render_fwd")):
        print(f"  {n.split('(')[0][:48]:48s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us  min {float(r['MinNs'])/1e3:8.1f}  max {float(r['MaxNs'])/1e3:8.1f}")
PY
done
