# round 5: kernel trace of lm_step (configs[2], val_batch 8) -- per-dispatch start / end for a timeline of the line search
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d /tmp/lt -o run -- python3 $GRAFT_REPO_ROOT/tools/exp/lm_phases.py --reps 1 > $GRAFT_REPO_ROOT/$O/lm.json 2> $GRAFT_REPO_ROOT/$O/lm.err || { tail -5 $GRAFT_REPO_ROOT/$O/lm.err; exit 1; }
f=$(find /tmp/lt -name "*kernel_trace.csv" | head -1)
echo "trace: $f"
gzip -c $f > $GRAFT_REPO_ROOT/$O/kernel_trace.csv.gz
tail -c 600 $GRAFT_REPO_ROOT/$O/lm.json
