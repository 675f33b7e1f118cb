# round 5: VJP hit loop over the batch's hit words (no HitIter) + record planes read from one address: GPU suite,
# A/B against HEAD (mv_ab stages, union stages), then the multi-stream raster sweep (r05u)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
TAG=r05v bash tools/exp/fwd2_ab.sh
bash tools/exp/r05u.sh
