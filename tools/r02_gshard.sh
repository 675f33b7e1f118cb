#!/bin/bash
# Gaussian-sharded exchange on the GPU: parity tests (2 processes on the one GPU, gloo-staged collectives) and a
# 2-rank bench rehearsal (GSLM_BENCH_DIST=gloo) of the N > 1 path
set -o pipefail
OUT=gpurun_out/r02b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_gshard.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|Error|assert" $OUT/tests.log | tail -30
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
GSLM_BENCH_DIST=gloo timeout -k 10 300 python bench.py --gpus 2 --P 200000 --steps 5 --warmup 2 --no-cpu-baseline \
  > $OUT/bench2.json 2> $OUT/bench2.err
rc2=$?
tail -5 $OUT/bench2.err
cut -c1-600 $OUT/bench2.json
exit $(( rc > rc2 ? rc : rc2 ))
