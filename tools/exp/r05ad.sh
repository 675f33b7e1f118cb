# round 5: two-launch scans (the apply pass sums its block's prefix of block sums; no single-block top scan) and the
# tile ranges zeroed by the duplicate kernels (no memset launch): GPU
# suite, A/B against HEAD (forward, union stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
TAG=r05ad bash tools/exp/fwd2_ab.sh
