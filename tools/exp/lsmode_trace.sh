# kernel traces of lm_phases.py with the per-set (0) and all-sets (1) line-search blends
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/lsmode
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in 0 1; do
  GSLM_LOSS_SET_GROUP=$m timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/t$m -o run -- python -u $GRAFT_REPO_ROOT/tools/exp/lm_phases.py --reps 2 > $GRAFT_REPO_ROOT/$O/t$m.json 2> $GRAFT_REPO_ROOT/$O/t$m.err || { echo "trace $m failed"; tail -5 $GRAFT_REPO_ROOT/$O/t$m.err; exit 1; }
  cat $GRAFT_REPO_ROOT/$O/t$m.json
done
