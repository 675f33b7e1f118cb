# round 6 call i: the drop-in backward memo for equal cotangents -- its GPU test, then the drop-in ops' profile with
# the memo on and off
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin_memo.py tests/test_gpu_dropin_branches.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for m in 1 0; do
  GSLM_BWD_MEMO=$m timeout -k 10 300 python tools/exp/dropin_prof.py > $O/dropin_prof_memo$m.log 2>&1 || { tail -20 $O/dropin_prof_memo$m.log; exit 1; }
  cp gpurun_out/dropin_prof.json $O/dropin_prof_memo$m.json
  grep -o '^[a-z_T]* {"ms": [0-9.]*' $O/dropin_prof_memo$m.log
done
