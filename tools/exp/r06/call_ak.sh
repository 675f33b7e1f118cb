# round 6 call ak: the tangent kernel held to 5 waves per SIMD (v_tangent_5w.py; 96 VGPRs, 80 B/lane of spills)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06ak build_head build_t5 build_head build_t5 > gpurun_out/r06ak.log 2>&1 || { tail -20 gpurun_out/r06ak.log; exit 1; }
for f in gpurun_out/r06ak/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'tangent_ms', 'render_matvec_loop_ms', 'gather_ms')})"; done
grep "equal" gpurun_out/r06ak.log | head -3
