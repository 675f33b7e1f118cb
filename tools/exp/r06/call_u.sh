# round 6 call u: the tangent kernel with its chain replaced by a 24-float linear map (timing floor, v_tfloor.py), and the gather with its chain replaced likewise (v_gfloor.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06u build build_tfloor build_gfloor build build_tfloor build_gfloor > gpurun_out/r06u.log 2>&1 || { tail -20 gpurun_out/r06u.log; exit 1; }
for f in gpurun_out/r06u/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06u.log | head -4
