#!/bin/bash
# A/B of one library build under environment switches: bash tools/env_ab.sh <tag> "<ENV=a>" "<ENV=b>" ...
# (each argument is an environment assignment list for one run of tools/mv_ab.py; runs in the given order)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for E in "$@"; do
  i=$((i + 1))
  name=$(echo "$E" | tr ' =' '__')
  env $E timeout -k 10 240 python tools/mv_ab.py "$name" --out /tmp/gslm_ab $MVAB_ARGS > $OUT/$i.$name.json 2> $OUT/$i.$name.err \
    || { tail -5 $OUT/$i.$name.err; exit 1; }
done
python tools/ab_summary.py $OUT
