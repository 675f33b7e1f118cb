# round 6 call aa: the LM tangent chain specialised without means tangents (v_tangent_nomeans.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06aa build build_tnm build build_tnm > gpurun_out/r06aa.log 2>&1 || { tail -20 gpurun_out/r06aa.log; exit 1; }
for f in gpurun_out/r06aa/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06aa.log | head -4
