# round 6 call p: nontemporal stores for the CG loop's streamed outputs (timing-only variant v_nt.py) against the tree
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06p build build_nt build build_nt > gpurun_out/r06p.log 2>&1 || { tail -20 gpurun_out/r06p.log; exit 1; }
for f in gpurun_out/r06p/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06p.log | head -4
