# round 5: the union rects folded into the line search's depth-space preprocess (gslm_preprocess_views_union +
# gslm_union_scan, ABI 10) -- line-search / LM-step tests, then lm_step against the HEAD package (ab_head/), alternated
set -o pipefail
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_line_search.py tests/test_gpu_lm_step.py -v -s --timeout 300 \
  --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for L in head new; do
    if [ $L = head ]; then export GSLM_PKG_DIR=$PWD/ab_head; else unset GSLM_PKG_DIR; fi
    timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_${L}_$r.json 2> $O/lm_${L}_$r.err \
      || { echo "lm_phases $L failed"; tail -5 $O/lm_${L}_$r.err; exit 1; }
    echo "$L r=$r $(cat $O/lm_${L}_$r.json)"
  done
done
