#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02d
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_lm.py tests/test_gpu_configs34.py -v -s --timeout 600 --timeout-method thread \
  > $OUT/tests.log 2>&1
rc=$?
grep -E "PASS|FAIL|passed|failed|Error|assert|drift" $OUT/tests.log | tail -30
exit $rc
