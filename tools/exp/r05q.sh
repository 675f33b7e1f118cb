# round 5: what bounds k_preprocess_views in depth space (scattered vs coalesced record writes)
set -o pipefail
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 300 python -u tools/exp/prev_writes.py --reps 10 > $O/prev.json 2> $O/prev.err || { tail -5 $O/prev.err; exit 1; }
cat $O/prev.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/pq -o run -- python3 $GRAFT_REPO_ROOT/tools/exp/prev_writes.py --reps 5 > /dev/null 2>&1 || exit 1
f=$(find /tmp/pq -name "*kernel_stats.csv" | head -1)
cp $f $GRAFT_REPO_ROOT/$O/kstats.csv
cd $GRAFT_REPO_ROOT
timeout -k 10 120 ./tools/exp/rp/rp_sort > $O/rp_sort.json && cat $O/rp_sort.json
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d /tmp/rq -o run -- $GRAFT_REPO_ROOT/tools/exp/rp/rp_sort > /dev/null 2>&1 || exit 1
f=$(find /tmp/rq -name "*kernel_stats.csv" | head -1)
cp $f $GRAFT_REPO_ROOT/$O/rp_kstats.csv
