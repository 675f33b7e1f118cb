# round 5: the line-search test with a batch above 8 views, then lm_step at val_batch 8 / 12 / 16 (chunked
# preprocesses) alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ao
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_line_search.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
BLIST="8 12 16 6" bash tools/exp/r05ak.sh
