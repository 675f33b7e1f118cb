#!/bin/bash
# SQ counters of one kernel for library builds: bash tools/sq_ab.sh <tag> <kernel regex> <build_dir>...
set -o pipefail
TAG=$1; RE=$2; shift 2
export TMPDIR=/tmp
ROOT=$(pwd)
for L in "$@"; do
  OUT=gpurun_out/$TAG/$L
  mkdir -p $OUT
  run() {
    local name=$1; shift
    (cd /tmp && GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -s KILL 120 rocprofv3 --pmc "$@" \
       --kernel-include-regex "$RE" -f csv -d "$ROOT/$OUT/$name" -o run -- python3 "$ROOT/tools/mv_ab.py" $L --reps 3 \
       --out /tmp/gslm_ab > /dev/null 2> "$ROOT/$OUT/$name.err")
  }
  run p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  && run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD \
  && echo "== $L" && python tools/sq_summary.py $OUT || exit 1
done
