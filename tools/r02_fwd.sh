#!/bin/bash
set -o pipefail
bash tools/ab_run.sh ab_fwd build_prev build || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_raster.py tests/test_gpu_fullsize.py tests/test_gpu_cull.py \
  tests/test_gpu_dropin_branches.py tests/test_gpu_batch_render.py -q --timeout 300 --timeout-method thread \
  > gpurun_out/fwd_tests.log 2>&1
rc=$?
tail -3 gpurun_out/fwd_tests.log
exit $rc
