#!/bin/bash
# round-2 first GPU call: the new parity tests (no -x: every failure is reported) then one bench line
set -o pipefail
OUT=gpurun_out/r02a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin_branches.py tests/test_gpu_batch_render.py \
  tests/test_gpu_lm_step.py tests/test_gpu_lm.py tests/test_gpu_knn.py -v --timeout 120 --timeout-method thread \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "passed|failed|Error|assert" $OUT/tests.log | tail -40
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc2=$?
tail -3 $OUT/bench.err
cat $OUT/bench.json
exit $rc2
