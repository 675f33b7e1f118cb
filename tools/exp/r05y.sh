# round 5: the final point through the kept union lists vs its exact render, wall and kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y
mkdir -p $O
timeout -k 10 300 python -u tools/exp/final_eval.py > $O/fe.json 2> $O/fe.err || { tail -5 $O/fe.err; exit 1; }
cat $O/fe.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/fe -o run -- python3 $GRAFT_REPO_ROOT/tools/exp/final_eval.py --reps 2 > /dev/null 2> $GRAFT_REPO_ROOT/$O/prof.err || { tail -5 $GRAFT_REPO_ROOT/$O/prof.err; exit 1; }
cp $(find /tmp/fe -name "*kernel_stats.csv" | head -1) $GRAFT_REPO_ROOT/$O/kstats.csv
gzip -c $(find /tmp/fe -name "*kernel_trace.csv" | head -1) > $GRAFT_REPO_ROOT/$O/trace.csv.gz
