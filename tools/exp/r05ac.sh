# round 5: k_ranges on 4 keys per thread and k_tile_order's wave scans: GPU suite, A/B against HEAD (forward, union
# stages), then the multi-rank rehearsals (tools/exp/r05ab.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ac
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
TAG=r05ac bash tools/exp/fwd2_ab.sh
bash tools/exp/r05ab.sh
