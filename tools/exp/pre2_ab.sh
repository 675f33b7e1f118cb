#!/bin/bash
# A/B of the preprocess's SH-rest staging (GSLM_PREPROCESS_STAGING=1: one 46-KB window; default: two windows), one
# build, both orders, with tools/mv_ab.py; then the products and images compared.  bash tools/exp/pre2_ab.sh <tag>
set -o pipefail
TAG=${1:-pre2_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for t in two one two2 one2; do
  case $t in one*) E=1 ;; *) E=2 ;; esac
  GSLM_PREPROCESS_STAGING=$E timeout -k 10 240 python tools/mv_ab.py $t --reps 30 --out /tmp/gslm_ab > $OUT/$t.json 2> $OUT/$t.err \
    || { tail -5 $OUT/$t.err; exit 1; }
  cat $OUT/$t.json; echo
done
python tools/mv_ab.py --compare /tmp/gslm_ab one two one2 two2 | tee $OUT/compare.txt
