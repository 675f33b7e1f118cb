# round 5: new GPU tests (NaN failure detection, SH degree 0/1 line search) + the LM tile cost order A/B
set -o pipefail
mkdir -p gpurun_out/r05b
timeout -k 10 400 python -u -m pytest tests/test_gpu_lm_step.py tests/test_gpu_line_search.py tests/test_gpu_lm.py -x -v \
  --timeout 120 --timeout-method thread > gpurun_out/r05b/gpu_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/r05b/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r05b/gpu_tests.log
MVAB_ARGS="--reps 40" bash tools/ab_run.sh r05b_ab build_base build build_base build
