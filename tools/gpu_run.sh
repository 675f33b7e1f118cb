#!/bin/bash
# One gpurun call: selected GPU tests, then bench.py, outputs under gpurun_out/$TAG.
#   gpurun -- 'TAG=r03a KEXPR="lm_step or rccl" bash tools/gpu_run.sh'   (TESTS=none: bench only; BENCH=0: tests only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-run}
mkdir -p gpurun_out/$TAG
if [ "${TESTS:-}" != "none" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread ${KEXPR:+-k "$KEXPR"} \
    > gpurun_out/$TAG/gpu_tests.log 2>&1 || { echo "gpu tests failed: $?"; tail -30 gpurun_out/$TAG/gpu_tests.log; exit 1; }
  tail -3 gpurun_out/$TAG/gpu_tests.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-600} python -u bench.py ${BENCH_ARGS:---steps 20 --warmup 5} > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err \
    || { echo "bench failed: $?"; tail -30 gpurun_out/$TAG/bench.err; exit 1; }
  cat gpurun_out/$TAG/bench.json
fi
