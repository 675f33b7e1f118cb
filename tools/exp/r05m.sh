# round 5: the tangent kernel's NOXYZ / PROJ instantiations and the batched ordered preprocess of the line search's
# final point (ABI 10) -- the whole GPU suite, then CG-loop and LM-step A/B against HEAD (ab_head/)
set -o pipefail
O=gpurun_out/r05m
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
    GSLM_LIB=$LIB GSLM_ABI_ANY=1 timeout -k 10 300 python -u tools/mv_ab.py $L --reps 40 --out /tmp/ab > $O/ab_${L}_$r.json \
      2> $O/ab_${L}_$r.err || { echo "mv_ab $L failed"; tail -5 $O/ab_${L}_$r.err; exit 1; }
    tail -c 400 $O/ab_${L}_$r.json; echo
    if [ $L = head ]; then export GSLM_PKG_DIR=$ROOT/ab_head; else unset GSLM_PKG_DIR; fi
    timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_${L}_$r.json 2> $O/lm_${L}_$r.err \
      || { echo "lm_phases $L failed"; tail -5 $O/lm_${L}_$r.err; exit 1; }
    unset GSLM_PKG_DIR
    echo "$L r=$r $(cat $O/lm_${L}_$r.json)"
  done
done
timeout -k 10 120 python -u tools/mv_ab.py --compare /tmp/ab head new
