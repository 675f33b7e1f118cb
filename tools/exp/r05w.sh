# round 5: the line search's final point through the kept union lists (gslm_union_extend, ABI 10): line-search and
# LM-step GPU tests, then lm_step phases (configs[2]) and the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_line_search.py tests/test_gpu_lm_step.py tests/test_cabi.py -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm.json 2> $O/lm.err || { tail -5 $O/lm.err; exit 1; }
tail -c 800 $O/lm.json
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['lm_step']['ms'], d['lm_step']['breakdown_ms'], d['lm_step'].get('exact_equal'), d['raster_streams']['ms_per_render'])"
