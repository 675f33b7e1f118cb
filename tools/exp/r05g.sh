# round 5: the whole GPU suite (drop-in backward: 8 waves per SIMD, visited rows after a zero fill, screen-position
# sums reduced and the conic applied per row); then kernel stats of the drop-in solver calls, fill vs no fill
set -o pipefail
O=gpurun_out/r05g
mkdir -p $O
ROOT=$PWD
export GSLM_MARGINS=$ROOT/$O/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head
case $rc in 0|1) ;; *) echo "test rc=$rc: stopping"; exit $rc;; esac
export TMPDIR=/tmp
for L in build_nofill build build_nofill build; do
  (cd /tmp && GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats \
     -f csv -d $ROOT/$O/prof_$L -o run -- python3 $ROOT/tools/exp/dropin_breakdown.py --reps 7 > $ROOT/$O/dropin_$L.json \
     2> $ROOT/$O/dropin_$L.err) || { echo "prof $L failed"; tail -5 $O/dropin_$L.err; exit 1; }
  cat $O/dropin_$L.json
  python - "$L" <<'PY'
import csv, sys
L = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/r05g/prof_{L}/run_kernel_stats.csv")):
    n = r["Name"].split("(")[0]
    if any(k in n for k in ("render_bwd", "preprocess_bwd", "fillBuffer")):
        print(f"  {L} {n[:50]:50s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us total {float(r['TotalDurationNs'])/1e6:7.2f} ms")
PY
done
