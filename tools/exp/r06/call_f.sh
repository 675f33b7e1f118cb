# round 6 call f: the benchmark-mode CG with the x update on a side stream (GSLM_CG_SIDE_X=1, default) against the
# in-place fused update (0): tests, mv_ab alternated on one library, then the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "side_stream or nocheck or cgls or drift or rccl or gshard or dist or lm_step" > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for m in 0 1; do
    GSLM_CG_SIDE_X=$m timeout -k 10 240 python tools/mv_ab.py side$m --reps 30 --out /tmp/gslm_ab > $O/mv_side${m}_r$r.json 2> $O/mv_side${m}_r$r.err || { tail -5 $O/mv_side${m}_r$r.err; exit 1; }
    cat $O/mv_side${m}_r$r.json
  done
done
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','forward_ms_per_view')}, d['cg_checked']['ms_per_step'], d['stage_ms'], d['lm_step']['ms'])"
