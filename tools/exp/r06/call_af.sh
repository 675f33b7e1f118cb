# round 6 call af: the forward's binning without k_tile_order, tiles blended in identity order (v_ident_order.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06af build_head build_io build_head build_io > gpurun_out/r06af.log 2>&1 || { tail -20 gpurun_out/r06af.log; exit 1; }
for f in gpurun_out/r06af/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06af.log | head -4
