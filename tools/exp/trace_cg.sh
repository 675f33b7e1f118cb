set -o pipefail
OUT=gpurun_out/r03s2_trace
mkdir -p $OUT
export TMPDIR=/tmp
ROOT=$(pwd)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $ROOT/$OUT -o run -- python3 $ROOT/bench.py --no-cpu-baseline --no-side --steps 20 --warmup 3 --forward-steps 8 > $ROOT/$OUT/bench.json 2> $ROOT/$OUT/err.log) \
&& python3 tools/exp/cg_trace.py $(find $OUT -name "*kernel_trace.csv" | head -1) > $OUT/cg_trace.txt && cat $OUT/cg_trace.txt \
&& python3 tools/trace_forward.py $(find $OUT -name "*kernel_trace.csv" | head -1) > $OUT/fwd.txt; cat $OUT/fwd.txt
