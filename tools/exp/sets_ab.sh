# all-sets blend at 8 waves per SIMD: line-search tests, union stages (fwd2_ab.sh) and the 50-view six-point timing
# per build (per-set and all-sets blends)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-sets_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "line_search or lm_step" > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/exp/fwd2_ab.sh
for L in build_base build; do
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 python -u tools/exp/ls_union.py --reps 3 --mode union > $O/ls_$L.json 2> $O/ls_$L.err || { echo "ls $L failed"; tail -5 $O/ls_$L.err; exit 1; }
  echo $L; cat $O/ls_$L.json
done
