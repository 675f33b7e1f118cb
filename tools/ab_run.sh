#!/bin/bash
# A/B timing of library builds with tools/mv_ab.py: bash tools/ab_run.sh <tag> <build_dir>...
# (build dirs under gaussian-splatting-lm_amd/, e.g. build build_x -- build revisions with tools/build_at.sh,
# which starts from an empty directory); then compares the products.  Extra mv_ab arguments: MVAB_ARGS.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for L in "$@"; do
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 python tools/mv_ab.py $L --out /tmp/gslm_ab $MVAB_ARGS \
    > $OUT/$L.json 2> $OUT/$L.err || { tail -5 $OUT/$L.err; exit 1; }
  cat $OUT/$L.json
done
python tools/mv_ab.py --compare /tmp/gslm_ab "$@"
