# round 6 call q: nontemporal stores for the gather y alone (v_nt_y.py) and the LM rows alone (v_nt_rows.py) against the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06q build build_nty build_ntr build build_nty build_ntr > gpurun_out/r06q.log 2>&1 || { tail -20 gpurun_out/r06q.log; exit 1; }
for f in gpurun_out/r06q/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06q.log | head -4
