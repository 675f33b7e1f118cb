# round 5: one-instruction scalar bookkeeping in the hit loops (clear_bit, live_update): GPU tests of the tile
# kernels, then A/B against HEAD (tools/exp/fwd2_ab.sh: mv_ab stages + forward, union-list stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
TAG=r05r bash tools/exp/fwd2_ab.sh
bash tools/ab_run.sh r05r_jvb build build_jvb build build_jvb > $O/ab_jvb.txt 2>&1 || { echo "ab jvb failed"; tail -20 $O/ab_jvb.txt; exit 1; }
tail -8 $O/ab_jvb.txt
