# round 6 call b: the GPU suite + bench on the tree (d11 depth sort, tightened bounds), then an A/B of the VJP
# barrier variants and the J v pin (tools/exp/r06/v_*.py; build_nosync is timing-only)
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r06b TEST_TIMEOUT=900 bash tools/gpu_run.sh || exit 1
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06b_ab build build_nostart build_nosync build_jvpin build > gpurun_out/r06b_ab.log 2>&1 || { tail -20 gpurun_out/r06b_ab.log; exit 1; }
cat gpurun_out/r06b_ab.log | grep -v "^\[" | tail -40
