#!/bin/bash
# SQ / GRBM counters of the tile passes (one PMC pass per counter group; no tracing domains).
#   bash tools/sq_counters.sh <tag> [kernel regex] [program: bench (default) | union]
# bench: bench.py's headline + forward (--no-side); union: tools/exp/union_kernels.py (the line search's union stages)
set -o pipefail
TAG=${1:-sq}
RE=${2:-k_render_matvec}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ROOT=$(pwd)
PROG="$ROOT/bench.py --no-cpu-baseline --no-side --steps 3 --warmup 1 --forward-steps 2"
[ "${3:-bench}" = "union" ] && PROG="$ROOT/tools/exp/union_kernels.py --reps 3"
run() {  # $1 = pass name, rest = counters
  local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -f csv -d "$ROOT/$OUT/$name" -o run \
     -- python3 $PROG > /dev/null 2> "$ROOT/$OUT/$name.err")
}
run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
&& run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD \
&& python tools/sq_summary.py "$OUT"
