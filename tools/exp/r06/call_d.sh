# round 6 call d: the window-claim VJP (vjp_tile_lm_async, build) against the batch VJP (build_sync, GSLM_VJP_ASYNC=0):
# mv_ab alternated with the products compared bitwise; the tangent kernel's geometry order (build_torig: after the
# direction update, build_tgl: parameter loads hoisted above it, build: geometry above it); then the GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06d_ab build_sync build build_sync build > gpurun_out/r06d_ab.log 2>&1 || { tail -30 gpurun_out/r06d_ab.log; exit 1; }
grep -v "^\[" gpurun_out/r06d_ab.log | tail -20
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06d_tab build_torig build_tgl build build_torig build_tgl build > gpurun_out/r06d_tab.log 2>&1 || { tail -30 gpurun_out/r06d_tab.log; exit 1; }
grep -v "^\[" gpurun_out/r06d_tab.log | grep tag
TAG=r06d TEST_TIMEOUT=900 BENCH=0 bash tools/gpu_run.sh
