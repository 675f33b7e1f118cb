# round 6 call r: nontemporal stores -- y (v_nt_y.py), y + x, y + x + s (v_nt_yx.py) against the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06r build build_nty build_ntyx build_ntyxs build build_nty build_ntyx build_ntyxs > gpurun_out/r06r.log 2>&1 || { tail -20 gpurun_out/r06r.log; exit 1; }
for f in gpurun_out/r06r/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06r.log | head -4
