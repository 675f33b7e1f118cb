# round 5: the drop-in backward's view-direction dot products formed block-cooperatively (tests + kernel stats against
# the HEAD build), the line search's kernels solo (val_batch 1: one stream) and at the default 8 streams, and the LM
# product as two launches (GSLM_MV_SPLIT) against the fused kernel
set -o pipefail
O=gpurun_out/r05j
mkdir -p $O
ROOT=$PWD
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin_branches.py tests/test_gpu_fullsize.py tests/test_gpu_raster.py \
  tests/test_gpu_edge.py tests/test_gpu_train.py -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 \
  || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for L in build_pbwd0 build build_pbwd0 build; do
  (cd /tmp && GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so GSLM_ABI_ANY=1 timeout -k 10 300 rocprofv3 --kernel-trace \
     --stats -f csv -d $ROOT/$O/dprof_$L -o run -- python3 $ROOT/tools/exp/dropin_breakdown.py --reps 7 \
     > $ROOT/$O/dropin_$L.json 2> $ROOT/$O/dropin_$L.err) || { echo "prof $L failed"; tail -5 $O/dropin_$L.err; exit 1; }
  cat $O/dropin_$L.json
  python3 - "$L" <<'PY'
import csv, sys
L = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/r05j/dprof_{L}/run_kernel_stats.csv")):
    n = r["Name"].split("(")[0]
    if any(k in n for k in ("render_bwd", "preprocess_bwd")):
        print(f"  {L} {n[:50]:50s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.1f} us")
PY
done
for vb in 1 8; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$O/vb$vb -o run -- \
     python3 $ROOT/tools/exp/lm_phases.py --reps 1 --val-batch $vb > $ROOT/$O/vb$vb.json 2> $ROOT/$O/vb$vb.err) \
     || { echo "vb $vb failed"; tail -5 $O/vb$vb.err; exit 1; }
  cat $O/vb$vb.json
  python3 - "$vb" <<'PY'
import csv, sys
vb = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/r05j/vb{vb}/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"vb {vb}: total kernel ms {tot/1e6:.1f}")
for r in rows[:22]:
    print(f"  {r['Calls']:>6s} {float(r['AverageNs'])/1e3:8.1f} {float(r['TotalDurationNs'])/1e6:8.2f}  {r['Name'][:90]}")
PY
done
# the LM product as two launches (GSLM_MV_SPLIT build) against the fused kernel, interleaved
for L in build build_split build build_split; do
  GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so GSLM_ABI_ANY=1 timeout -k 10 300 python -u tools/mv_ab.py $L \
    --reps 20 --out $O/ab > $O/ab_$L.json 2> $O/ab_$L.err || { echo "mv_ab $L failed"; tail -5 $O/ab_$L.err; exit 1; }
  tail -c 700 $O/ab_$L.json; echo
done
timeout -k 10 120 python -u tools/mv_ab.py --compare $O/ab build build_split
