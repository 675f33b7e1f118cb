# round 6 call ae: the key-range depth sort with the copy passes (build_dr) and with three-pair routing (build_dr3)
set -o pipefail
cd $GRAFT_REPO_ROOT
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_dr3/libgslm.so timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_depth_sort.py tests/test_gpu_raster.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py tests/test_gpu_configs34.py tests/test_gpu_line_search.py > gpurun_out/r06ae_tests.log 2>&1 || { tail -40 gpurun_out/r06ae_tests.log; exit 1; }
tail -2 gpurun_out/r06ae_tests.log
MVAB_ARGS="--reps 30" timeout -k 10 700 bash tools/ab_run.sh r06ae build_head build_dr build_dr3 build_head build_dr build_dr3 > gpurun_out/r06ae.log 2>&1 || { tail -20 gpurun_out/r06ae.log; exit 1; }
for f in gpurun_out/r06ae/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06ae.log | head -8
timeout -k 10 300 bash tools/prof_forward.sh build_head > gpurun_out/r06ae_tl_head.txt 2>&1 && timeout -k 10 300 bash tools/prof_forward.sh build_dr3 > gpurun_out/r06ae_tl_dr3.txt 2>&1
