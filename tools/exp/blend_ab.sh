# blend-kernel change: raster / cull / line-search tests, then A/B (tools/exp/fwd2_ab.sh: forward, union stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-blend_ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread -k "${KEXPR:-cull or line_search or lm_step or raster or fullsize or golden}" > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/exp/fwd2_ab.sh
