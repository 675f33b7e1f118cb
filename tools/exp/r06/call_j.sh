# round 6 call j: the configs[2] LM step in bench.py's line against tools/exp/lm_phases.py on the same box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python tools/exp/lm_phases.py --reps 5 > $O/lm_phases.json 2> $O/lm_phases.err || { tail -20 $O/lm_phases.err; exit 1; }
cat $O/lm_phases.json
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); l = d['lm_step']
print({k: l[k] for k in ('ms', 'ms_min', 'ms_max', 'breakdown_ms')}, d['ms_per_step'], d['forward_ms_per_view'], d['dropin_solver_ops'])"
timeout -k 10 300 python tools/exp/lm_phases.py --reps 5 > $O/lm_phases2.json 2> $O/lm_phases2.err || { tail -20 $O/lm_phases2.err; exit 1; }
cat $O/lm_phases2.json
