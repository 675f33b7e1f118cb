# round 5: where the drop-in solver ops' time goes on the final kernels (torch.profiler trace per op)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aa
mkdir -p $O
timeout -k 10 400 python -u tools/exp/dropin_prof.py > $O/dropin.json 2> $O/dropin.err || { tail -5 $O/dropin.err; exit 1; }
python3 -c "import json;print(json.dumps(json.loads(open('$O/dropin.json').read().strip().splitlines()[-1]), indent=1)[:6000])"
