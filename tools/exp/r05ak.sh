# round 5: lm_step's val_batch (views per batch of the line search: 4 / 6 / 8 = default / 12 / 16) with the evaluator's
# default 3 side streams; interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ak
mkdir -p $O
for r in 1 2; do
  for b in ${BLIST:-8 4 6 12 16}; do
    timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 --val-batch $b > $O/lm_b${b}_$r.json 2> $O/lm_b${b}_$r.err || { tail -5 $O/lm_b${b}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lm_b${b}_$r.json').read().strip().splitlines()[-1]);print('val_batch $b run $r', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
  done
done
