# round 5: the line search's blends per set (GSLM_LOSS_SETS=1) or all six per pass (6), each with the main-stream half
# on a default- or high-priority stream (GSLM_LS_HIPRI); lm_phases interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05af
mkdir -p $O
for r in 1 2; do
  for cfg in "1 0" "1 1" "6 0" "6 1"; do
    set -- $cfg
    GSLM_LOSS_SETS=$1 GSLM_LS_HIPRI=$2 timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_s$1_p$2_$r.json 2> $O/lm_s$1_p$2_$r.err || { tail -5 $O/lm_s$1_p$2_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lm_s$1_p$2_$r.json').read().strip().splitlines()[-1]);print('sets $1 hipri $2 run $r', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
  done
done
