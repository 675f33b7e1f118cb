# round 6 call ac: (fence-free form, v_hist_scan_ticket2.py) each radix pass's block scan folded into its histogram kernel via arrival tickets (v_hist_scan_ticket.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_hst2/libgslm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_fullsize.py tests/test_gpu_raster.py tests/test_gpu_edge.py > gpurun_out/r06ac_tests.log 2>&1 || { tail -30 gpurun_out/r06ac_tests.log; exit 1; }
tail -2 gpurun_out/r06ac_tests.log
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06ac build build_hst2 build build_hst2 > gpurun_out/r06ac.log 2>&1 || { tail -20 gpurun_out/r06ac.log; exit 1; }
for f in gpurun_out/r06ac/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06ac.log | head -6
