# round 5: r05m after the stream-order fix of the batched final-point preprocess
set -o pipefail
ROOT=$PWD
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_line_search.py tests/test_gpu_lm_step.py tests/test_gpu_lm.py -v -s \
  --timeout 300 --timeout-method thread > $O/tests_ls.log 2>&1 || { tail -30 $O/tests_ls.log; exit 1; }
tail -2 $O/tests_ls.log
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
