# hardware sqrt in the quadrant test: cull / line-search / raster tests, then A/B (forward, union stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-sqrt_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "cull or line_search or lm_step or raster or fullsize" > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
bash tools/exp/fwd2_ab.sh
