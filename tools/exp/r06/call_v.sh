# round 6 call v: k_dot_final as one 1024-thread block (v_dotfinal1024.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06v build build_df1024 build build_df1024 > gpurun_out/r06v.log 2>&1 || { tail -20 gpurun_out/r06v.log; exit 1; }
for f in gpurun_out/r06v/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06v.log | head -4
