# round 5: (1) the whole GPU suite on the tree with the paired VJP visits and the drop-in backward at 8 waves per SIMD
# (rows for visited entries only, no materialised inverse-depth gradient); (2) A/B paired vs single VJP visits;
# (3) the bench line (dropin_solver_ops, raster_fwd_bwd)
set -o pipefail
O=gpurun_out/r05e
mkdir -p $O
export GSLM_MARGINS=$PWD/$O/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head
case $rc in 0|1) ;; *) echo "test rc=$rc: stopping"; exit $rc;; esac
MVAB_ARGS="--reps 40" bash tools/ab_run.sh r05e_ab build_np build build_np build || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r05e/bench.json").read().strip().splitlines()[-1])
print(json.dumps({k: d.get(k) for k in ("value", "ms_per_step", "raster_mpix_s", "forward_ms_per_view", "stage_ms", "dropin_solver_ops", "raster_fwd_bwd", "lm_step")})[:2500])
PY
