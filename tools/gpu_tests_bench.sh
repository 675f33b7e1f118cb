#!/bin/bash
# GPU tests (given files, or all -m gpu) then one bench line: gpurun_out/<tag>/{tests.log,bench.json,bench.err}.
#   usage: bash tools/gpu_tests_bench.sh <tag> [test files...]
set -o pipefail
TAG=${1:-tb}
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
fi
rc=$?
tail -25 "$OUT/tests.log"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -3 "$OUT/bench.err"
cat "$OUT/bench.json"
exit $rc
