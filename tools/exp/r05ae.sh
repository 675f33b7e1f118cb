# round 5: the native communicators closed in order before the process group (RCCL / multi-rank GPU tests)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ae
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_dist.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
