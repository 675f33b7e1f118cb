#!/bin/bash
# A/B of the LM linearisation record (GSLM_LM_LREC=0: the per-product primal chains) with tools/mv_ab.py, one build,
# both orders; then the products compared.  bash tools/exp/lrec_ab.sh <tag>
set -o pipefail
TAG=${1:-lrec_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for t in on off on2 off2; do
  case $t in on*) E=1 ;; *) E=0 ;; esac
  GSLM_LM_LREC=$E timeout -k 10 240 python tools/mv_ab.py $t --out /tmp/gslm_ab > $OUT/$t.json 2> $OUT/$t.err \
    || { tail -5 $OUT/$t.err; exit 1; }
  cat $OUT/$t.json; echo
done
python tools/mv_ab.py --compare /tmp/gslm_ab off on off2 on2 | tee $OUT/compare.txt
