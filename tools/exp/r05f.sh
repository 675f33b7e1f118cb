# round 5: the drop-in backward (96-entry batches at 8 waves per SIMD, rows for visited entries only after a zero
# fill, no materialised inverse-depth gradient): its tests, then kernel stats of the drop-in solver calls
# (tools/exp/dropin_breakdown.py) for round 4's library and this tree
set -o pipefail
O=gpurun_out/r05f
mkdir -p $O
ROOT=$PWD
timeout -k 10 600 python -u -m pytest tests/test_gpu_cull.py tests/test_gpu_raster.py tests/test_gpu_dropin_branches.py \
  tests/test_gpu_edge.py tests/test_gpu_batch_render.py tests/test_gpu_train.py tests/test_gpu_fullsize.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head
case $rc in 0|1) ;; *) echo "test rc=$rc: stopping"; exit $rc;; esac
export TMPDIR=/tmp
for L in build_base build; do
  (cd /tmp && GSLM_ABI_ANY=1 GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -f csv -d $ROOT/$O/prof_$L -o run -- python3 $ROOT/tools/exp/dropin_breakdown.py --reps 7 > $ROOT/$O/dropin_$L.json \
     2> $ROOT/$O/dropin_$L.err) || { echo "prof $L failed"; tail -5 $O/dropin_$L.err; exit 1; }
  cat $O/dropin_$L.json
done
python - <<'PY'
import csv
for L in ("build_base", "build"):
    print(L)
    for r in csv.DictReader(open(f"gpurun_out/r05f/prof_{L}/run_kernel_stats.csv")):
        n = r["Name"].split("(")[0]
        if any(k in n for k in ("render_bwd", "preprocess_bwd", "render_jvp", "tangent", "fillBuffer")):
            print(f"  {n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
