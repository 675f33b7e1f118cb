#!/bin/bash
# A/B timing of library builds with tools/mv_ab.py: bash tools/ab_run.sh <tag> <build_dir>...
# (build dirs under gaussian-splatting-lm_amd/, e.g. build build_x -- build revisions with tools/build_at.sh,
# which starts from an empty directory); then compares the products.  Extra mv_ab arguments: MVAB_ARGS.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for L in "$@"; do
  i=$((i + 1))
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 python tools/mv_ab.py $L --out /tmp/gslm_ab $MVAB_ARGS \
    > $OUT/$i.$L.json 2> $OUT/$i.$L.err || { tail -5 $OUT/$i.$L.err; exit 1; }
  cat $OUT/$i.$L.json
done
python tools/mv_ab.py --compare /tmp/gslm_ab "$@"
