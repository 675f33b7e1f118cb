# round 6 call z: the VJP pass in 256-entry batches (v_batch256.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06z build build_b256 build build_b256 > gpurun_out/r06z.log 2>&1 || { tail -20 gpurun_out/r06z.log; exit 1; }
for f in gpurun_out/r06z/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06z.log | head -4
