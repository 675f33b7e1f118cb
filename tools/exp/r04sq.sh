# SQ / GRBM counters: the CG product and the forward blend (bench.py --no-side), then the union stages
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/sq_counters.sh r04sq_bench 'k_render' > gpurun_out/r04sq_bench.txt 2>&1 || { echo "bench sq failed"; tail -20 gpurun_out/r04sq_bench.txt; exit 1; }
bash tools/sq_counters.sh r04sq_union 'k_duplicate|k_radix_scatter|k_render_fwd_wave' union > gpurun_out/r04sq_union.txt 2>&1 || { echo "union sq failed"; tail -20 gpurun_out/r04sq_union.txt; exit 1; }
cat gpurun_out/r04sq_bench.txt gpurun_out/r04sq_union.txt
