# round 5: the whole GPU suite (new: NaN failure detection, debug mode, SH degree 0/1 line search, ABI 9 union checks,
# the stable-quantity CG bounds, the parity margin log) + the LM tile cost order A/B against round 4's library
set -o pipefail
mkdir -p gpurun_out/r05b
export GSLM_MARGINS=$PWD/gpurun_out/r05b/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/r05b/gpu_tests.log 2>&1
rc=$?
tail -3 gpurun_out/r05b/gpu_tests.log
grep -E "FAILED|ERROR" gpurun_out/r05b/gpu_tests.log | head -20
case $rc in 0|1) ;; *) echo "test run ended with rc=$rc: stopping"; exit $rc;; esac
MVAB_ARGS="--reps 40" bash tools/ab_run.sh r05b_ab build_base build build_base build
