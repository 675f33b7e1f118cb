# round 5: re-run the reworked parity bounds (model decrease, whole-frame L2) + the VJP prefetch A/B
set -o pipefail
mkdir -p gpurun_out/r05c
export GSLM_MARGINS=$PWD/gpurun_out/r05c/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 600 python -u -m pytest tests/test_gpu_drift.py tests/test_gpu_lm.py tests/test_gpu_fullsize.py -m gpu -v -s \
  --timeout 300 --timeout-method thread > gpurun_out/r05c/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05c/gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r05c/gpu_tests.log | head -20
case $rc in 0|1) ;; *) echo "test run ended with rc=$rc: stopping"; exit $rc;; esac
MVAB_ARGS="--reps 40" bash tools/ab_run.sh r05c_ab build_order build_pf build_pfe build_order build_pf build_pfe
