# round 6 call w: the line search's per-batch pair-count read-back as one gather launch into pinned memory (instead of
# a 4-byte copy per geometry) -- the line-search / LM-step GPU tests, then lm_phases alternated against HEAD's library
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "line_search or lm_step or evaluator or union or num_rendered" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  for L in build build_head; do
    GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 python tools/exp/lm_phases.py --reps 5 > $O/lm_${L}_r$r.json 2> $O/lm_${L}_r$r.err || { tail -5 $O/lm_${L}_r$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lm_${L}_r$r.json')); u=sorted(d['untimed_ms']); print('$L r$r', u[len(u)//2], u, [t['line_search_ms'] for t in d['timed']])"
  done
done
