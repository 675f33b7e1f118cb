# round 5: the validation evaluator's stream count (GSLM_VAL_STREAMS; NLIST, default 8 4 2 6) in lm_step; interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai
mkdir -p $O
for r in 1 2; do
  for n in ${NLIST:-8 4 2 6}; do
    GSLM_VAL_STREAMS=$n timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_s${n}_$r.json 2> $O/lm_s${n}_$r.err || { tail -5 $O/lm_s${n}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lm_s${n}_$r.json').read().strip().splitlines()[-1]);print('streams $n run $r', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
  done
done
