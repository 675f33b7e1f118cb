#!/bin/bash
# One measurement call on the MI355X box (run through gpurun from the repo root):
#   GPU tests -> bench line -> rocprofv3 kernel stats -> separate FETCH_SIZE / WRITE_SIZE PMC passes.
# Every GPU step has its own time limit and the steps are chained with &&: the first failure ends
# the call (nothing is retried).  Outputs land in gpurun_out/<tag>/; copy the summaries you want
# judged into profiles/<round>/.
#   usage: bash tools/gpu_profile.sh <tag> [tests|notests] [bench args...]
set -o pipefail
TAG=${1:-run}
MODE=${2:-tests}
[ $# -ge 2 ] && shift 2 || shift $#
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
PROFARGS="--no-cpu-baseline --steps 10 --warmup 3 --forward-steps 8 $*"
# the headline and the forward alone (no side measurements: one stream, no line-search overlap in the kernel averages)
SOLOARGS="$PROFARGS --no-side"

step_tests() {
  if [ "$MODE" = "tests" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
  fi
}

step_tests \
&& timeout -k 10 600 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" \
&& (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/stats" -o run \
      -- python3 "$ROOT/bench.py" $PROFARGS > "$ROOT/$OUT/prof_bench.json" 2> "$ROOT/$OUT/prof.err") \
&& (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/stats_solo" -o run \
      -- python3 "$ROOT/bench.py" $SOLOARGS > "$ROOT/$OUT/prof_bench_solo.json" 2> "$ROOT/$OUT/prof_solo.err") \
&& (cd /tmp && timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -f csv -d "$ROOT/$OUT/pmc_fetch" -o run \
      -- python3 "$ROOT/bench.py" $SOLOARGS > /dev/null 2> "$ROOT/$OUT/pmc_fetch.err") \
&& (cd /tmp && timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -f csv -d "$ROOT/$OUT/pmc_write" -o run \
      -- python3 "$ROOT/bench.py" $SOLOARGS > /dev/null 2> "$ROOT/$OUT/pmc_write.err") \
&& python tools/pmc_summary.py "$OUT" "$OUT/pmc_render_matvec.json" > "$OUT/pmc_summary.json"
rc=$?
echo "exit $rc"
cat "$OUT/bench.json" 2>/dev/null
tail -3 "$OUT/gpu_tests.log" 2>/dev/null
exit $rc
