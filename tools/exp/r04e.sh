# line-search tests, the union timing tool, then its kernel-trace profile (csv)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -rP -k "${KEXPR:-line_search or lm_step}" > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
timeout -k 10 300 python -u tools/exp/ls_union.py --reps 3 > $O/ls.json 2> $O/ls.err || { echo "ls failed"; tail -20 $O/ls.err; exit 1; }
cat $O/ls.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python -u $GRAFT_REPO_ROOT/tools/exp/ls_union.py --reps 2 --mode union > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { echo "prof failed"; tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*stats*"
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/exp/dropin_breakdown.py > $O/dropin.json 2> $O/dropin.err || { echo "dropin failed"; tail -20 $O/dropin.err; exit 1; }
cat $O/dropin.json
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
  cat $O/bench.json
fi
