# Full GPU suite, then an A/B of library builds (tools/ab_run.sh), in one gpurun call:
#   gpurun -- 'TAG=r03s3_x bash tools/exp/run_compact.sh build_base build build_base build'
set -o pipefail
TAG=${TAG:-tests_ab}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|assert" $O/gpu_tests.log | head -30; tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/ab_run.sh ${TAG}_ab "$@"
