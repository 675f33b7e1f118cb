# round 6 call aj: the line search blends per set (GSLM_LOSS_SET_GROUP=1, the default) against groups of 2 and 3 sets per
# pass over the union list inside lm_step at the shipped evaluator setting (3 side streams), alternated twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06aj
mkdir -p $O
for r in 1 2; do
  for k in 1 2 3; do
    GSLM_LOSS_SET_GROUP=$k timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 5 > $O/lm_k${k}_r$r.json 2> $O/lm_k${k}_r$r.err \
      || { echo "lm_phases k=$k failed"; tail -5 $O/lm_k${k}_r$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/lm_k${k}_r$r.json')); u=sorted(d['untimed_ms']); print('k=$k r=$r untimed median', u[len(u)//2], u)"
  done
done
