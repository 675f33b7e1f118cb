# round 6 call x: k_gather_lm at 7 and 8 waves per SIMD (v_gather_lb7.py, v_gather_lb8.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06x build build_glb7 build_glb8 build build_glb7 build_glb8 > gpurun_out/r06x.log 2>&1 || { tail -20 gpurun_out/r06x.log; exit 1; }
for f in gpurun_out/r06x/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"; done
grep "equal=" gpurun_out/r06x.log | head -4
