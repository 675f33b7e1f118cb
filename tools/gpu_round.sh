#!/bin/bash
# Full GPU suite, the bench line, and the multi-rank rehearsals (gloo 2 ranks on one GPU; one-rank RCCL), one call:
#   gpurun -- 'TAG=r03m bash tools/gpu_round.sh'
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-round}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 \
  || { echo "gpu tests failed: $?"; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
  || { echo "bench failed: $?"; tail -30 $O/bench.err; exit 1; }
head -c 400 $O/bench.json; echo
GSLM_BENCH_DIST=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "gloo2 failed: $?"; tail -30 $O/bench_gloo2.err; exit 1; }
head -c 400 $O/bench_gloo2.json; echo
GSLM_FORCE_COLLECTIVES=1 GSLM_BENCH_EXCHANGE=gaussian timeout -k 10 600 python -u bench.py --no-cpu-baseline \
  > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { echo "rccl1 failed: $?"; tail -30 $O/bench_rccl1.err; exit 1; }
head -c 400 $O/bench_rccl1.json; echo
