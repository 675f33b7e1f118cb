# round 6 call ai: the LM VJP batches over the head entries only (ScratchBufs::hsort / hlist; working tree -> build_hd)
set -o pipefail
cd $GRAFT_REPO_ROOT
export GSLM_MARGINS=gpurun_out/r06ai/parity_margins.jsonl
mkdir -p gpurun_out/r06ai
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_hd/libgslm.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06ai_tests.log 2>&1 || { tail -40 gpurun_out/r06ai_tests.log; exit 1; }
tail -1 gpurun_out/r06ai_tests.log
unset GSLM_MARGINS
MVAB_ARGS="--reps 30" timeout -k 10 700 bash tools/ab_run.sh r06ai_ab build_head build_hd build_head build_hd > gpurun_out/r06ai.log 2>&1 || { tail -20 gpurun_out/r06ai.log; exit 1; }
for f in gpurun_out/r06ai_ab/*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(d[k], 4) for k in ('cg_iter_ms', 'forward_ms', 'render_matvec_loop_ms')})"; done
grep "equal" gpurun_out/r06ai.log | head -4
