# round 5: the validation evaluator's side streams (binnings + blends) at high priority (GSLM_SIDE_HIPRI=1) against the
# default; lm_phases interleaved three times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag
mkdir -p $O
for r in 1 2 3; do
  for p in 0 1; do
    GSLM_SIDE_HIPRI=$p timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_p${p}_$r.json 2> $O/lm_p${p}_$r.err || { tail -5 $O/lm_p${p}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lm_p${p}_$r.json').read().strip().splitlines()[-1]);print('side hipri $p run $r', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
  done
done
