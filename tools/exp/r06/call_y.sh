# round 6 call y: the LM VJP pass with wave-private staging and a last-arriver combine, 64- and 32-entry windows (v_vjp_private.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06y build build_vp64 build_vp32 build build_vp64 build_vp32 > gpurun_out/r06y.log 2>&1 || { tail -20 gpurun_out/r06y.log; exit 1; }
for f in gpurun_out/r06y/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06y.log | head -12
