# round 6 call ad: the depth sort over the frame's key span (sort.hip KeyRange; working tree built into build_dr)
set -o pipefail
cd $GRAFT_REPO_ROOT
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_dr/libgslm.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_depth_sort.py tests/test_gpu_raster.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py tests/test_gpu_configs34.py > gpurun_out/r06ad_tests.log 2>&1 || { tail -40 gpurun_out/r06ad_tests.log; exit 1; }
tail -2 gpurun_out/r06ad_tests.log
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06ad build_head build_dr build_head build_dr > gpurun_out/r06ad.log 2>&1 || { tail -20 gpurun_out/r06ad.log; exit 1; }
for f in gpurun_out/r06ad/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06ad.log | head -6
