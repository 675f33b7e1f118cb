# round 5: A/B of the final point through the kept union lists (GSLM_LS_FINAL=union, default) against its exact render
# (GSLM_LS_FINAL=exact): lm_phases interleaved twice, then the bench's lm_step row each way
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05x
mkdir -p $O
for r in 1 2; do
  for f in exact union; do
    GSLM_LS_FINAL=$f timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_${f}_$r.json 2> $O/lm_${f}_$r.err || { tail -5 $O/lm_${f}_$r.err; exit 1; }
    echo "$f $r $(tail -c 420 $O/lm_${f}_$r.json)"
  done
done
