# round 5: the balance-preserving XCD-aware length order (k_tile_order_xcdl) for the forward and the loss blends,
# against the frame-wide one (GSLM_LEN_ORDER=flat): GPU suite, then mv_ab / union stages / lm_phases alternated
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05aq
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
for r in 1 2; do
  for m in flat xcdl; do
    GSLM_LEN_ORDER=$m timeout -k 10 240 python tools/mv_ab.py $m --out /tmp/ab_aq > $O/mv_${m}_$r.json 2> $O/mv_${m}_$r.err || { tail -5 $O/mv_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/mv_${m}_$r.json').read().strip().splitlines()[-1]);print('$m $r', {k:round(v,4) for k,v in d.items() if k in ('cg_iter_ms','render_matvec_ms','forward_ms')})"
    GSLM_LEN_ORDER=$m timeout -k 10 240 python -u tools/exp/union_kernels.py > $O/uk_${m}_$r.json 2> $O/uk_${m}_$r.err || { tail -5 $O/uk_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/uk_${m}_$r.json').read().strip().splitlines()[-1]);print('  uk $m', round(d['blends_6_slot_ms'],4), round(d['union_binning_ms'],4), round(d['exact_6_points_ms'],4))"
  done
done
python tools/mv_ab.py --compare /tmp/ab_aq flat xcdl
for m in flat xcdl flat xcdl; do
  GSLM_LEN_ORDER=$m timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_$m.json 2> $O/lm_$m.err || { tail -5 $O/lm_$m.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/lm_$m.json').read().strip().splitlines()[-1]);print('lm $m', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
done
