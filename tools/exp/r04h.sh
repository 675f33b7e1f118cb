# the union-list stages of one view on one stream, plus a kernel-stats profile of the same
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04h}
mkdir -p $O
timeout -k 10 300 python -u tools/exp/union_kernels.py > $O/uk.json 2> $O/uk.err || { echo "uk failed"; tail -20 $O/uk.err; exit 1; }
cat $O/uk.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python -u $GRAFT_REPO_ROOT/tools/exp/union_kernels.py --reps 3 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
