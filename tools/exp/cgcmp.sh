set -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
mkdir -p gpurun_out/cgcmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $ROOT/gpurun_out/cgcmp/b -o run -- python3 $ROOT/bench.py --no-cpu-baseline --steps 10 --warmup 3 --forward-steps 2 > $ROOT/gpurun_out/cgcmp/b.json 2>/dev/null) \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $ROOT/gpurun_out/cgcmp/m -o run -- python3 $ROOT/tools/mv_ab.py x --reps 10 --cg-scan 10 > $ROOT/gpurun_out/cgcmp/m.json 2>/dev/null) \
&& python3 tools/exp/cg_trace.py $(find gpurun_out/cgcmp/b -name "*kernel_trace.csv" | head -1) bench \
&& python3 tools/exp/cg_trace.py $(find gpurun_out/cgcmp/m -name "*kernel_trace.csv" | head -1) mvab
