# round 6 call o: the dot finalisations fused into their producers' last block (ABI 10) -- GPU tests of the CG paths,
# then mv_ab with GSLM_DOT_LASTBLOCK=1 / 0 alternated twice (0: the separate finalisation launches)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "last_block or cgls or recursions or lm_step or drift" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for m in 1 0; do
    GSLM_DOT_LASTBLOCK=$m timeout -k 10 240 python tools/mv_ab.py lb$m --reps 30 --out /tmp/gslm_ab > $O/mv_lb${m}_r$r.json 2> $O/mv_lb${m}_r$r.err || { tail -5 $O/mv_lb${m}_r$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/mv_lb${m}_r$r.json')); print('lb$m r$r', {k: round(d[k], 4) for k in ('cg_iter_ms', 'render_matvec_loop_ms', 'gather_ms', 'tangent_ms')})"
  done
done
