# round 5: HIP hardware queues per process (GPU_MAX_HW_QUEUES: the box default 4, then 8 and 16) for the LM step's
# 9 streams (lm_phases) and bench.py's 8-stream raster; interleaved twice
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah
mkdir -p $O
for r in 1 2; do
  for q in 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_q${q}_$r.json 2> $O/lm_q${q}_$r.err || { tail -5 $O/lm_q${q}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/lm_q${q}_$r.json').read().strip().splitlines()[-1]);print('queues $q run $r', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
  done
done
for q in 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/bench_q$q.json 2> $O/bench_q$q.err || { tail -5 $O/bench_q$q.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_q$q.json').read().strip().splitlines()[-1]);print('queues $q bench', d['value'], d['raster_mpix_s'], d['raster_streams']['ms_per_render'], d['lm_step']['ms'])"
done
