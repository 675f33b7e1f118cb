# round 6 call ag: the forward blend as one 64-thread block per (tile, quadrant) (v_fwd_wave_blocks.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_wb/libgslm.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_raster.py tests/test_gpu_edge.py > gpurun_out/r06ag_tests.log 2>&1 || { tail -30 gpurun_out/r06ag_tests.log; exit 1; }
tail -1 gpurun_out/r06ag_tests.log
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06ag build_head build_wb build_head build_wb > gpurun_out/r06ag.log 2>&1 || { tail -20 gpurun_out/r06ag.log; exit 1; }
for f in gpurun_out/r06ag/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06ag.log | head -4
