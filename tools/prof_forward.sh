#!/bin/bash
# kernel trace of tools/mv_ab.py for one library build and the last forward's timeline
set -o pipefail
L=${1:-build}
OUT=gpurun_out/proff_$L
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv \
   -d $ROOT/$OUT -o run -- python3 $ROOT/tools/mv_ab.py $L --reps 5 > $ROOT/$OUT/ab.json 2> $ROOT/$OUT/err.log) || exit 1
python3 tools/trace_forward.py $(find $OUT -name "*kernel_trace.csv" | head -1)
