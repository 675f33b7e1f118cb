# round 6 call h: where the drop-in solver ops' time goes on the current tree (torch.profiler table per op)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp/dropin_prof.py > $O/dropin_prof.log 2>&1 || { tail -20 $O/dropin_prof.log; exit 1; }
cp gpurun_out/dropin_prof.json $O/
tail -5 $O/dropin_prof.log
