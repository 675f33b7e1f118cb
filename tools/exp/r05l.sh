# round 5: VJP visit trims (the unused reduction slot paired with a dead register; the conic / screen-position rows'
# opacity factor applied once per row at the combine) -- the whole GPU suite, then the CG-loop A/B against HEAD's
# library (ab_head/build) and the drop-in breakdown
set -o pipefail
O=gpurun_out/r05l
mkdir -p $O
ROOT=$PWD
export GSLM_MARGINS=$ROOT/$O/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
case $rc in 0) ;; *) echo "test rc=$rc: stopping"; exit $rc;; esac
for r in 1 2; do
  for L in head new; do
    if [ $L = head ]; then LIB=$ROOT/ab_head/build/libgslm.so; else LIB=$ROOT/gaussian-splatting-lm_amd/build/libgslm.so; fi
    GSLM_LIB=$LIB GSLM_ABI_ANY=1 timeout -k 10 300 python -u tools/mv_ab.py $L --reps 40 --out $O/ab > $O/ab_${L}_$r.json \
      2> $O/ab_${L}_$r.err || { echo "mv_ab $L failed"; tail -5 $O/ab_${L}_$r.err; exit 1; }
    tail -c 400 $O/ab_${L}_$r.json; echo
  done
done
timeout -k 10 120 python -u tools/mv_ab.py --compare $O/ab head new
timeout -k 10 300 python -u tools/exp/dropin_breakdown.py --reps 7 > $O/dropin.json 2> $O/dropin.err && cat $O/dropin.json
