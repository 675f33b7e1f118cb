# round 5: SQ counters of the blends (forward k_render_fwd_wave<0> from bench.py, line-search slot blends from
# union_kernels.py) on the tree with the one-instruction hit-loop bookkeeping
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/sq_counters.sh r05s_fwd k_render_fwd_wave bench > gpurun_out/r05s_fwd.txt 2>&1 || { tail -5 gpurun_out/r05s_fwd.txt; exit 1; }
cat gpurun_out/r05s_fwd.txt
bash tools/sq_counters.sh r05s_union "k_render_fwd_wave|k_duplicate_union|k_union_rect|k_radix" union > gpurun_out/r05s_union.txt 2>&1 || { tail -5 gpurun_out/r05s_union.txt; exit 1; }
cat gpurun_out/r05s_union.txt
