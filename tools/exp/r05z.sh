# round 5 final tree: GPU suite, bench line, rocprof kernel stats (bench + solo), FETCH/WRITE PMC passes, SQ counters
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile.sh r05z tests || exit 1
bash tools/sq_counters.sh r05z_sq k_render_matvec bench > gpurun_out/r05z_sq.txt 2>&1 || { tail -5 gpurun_out/r05z_sq.txt; exit 1; }
cat gpurun_out/r05z_sq.txt | head -40
