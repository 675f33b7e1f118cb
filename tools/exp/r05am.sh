# round 5: the XCD-aware order for the LM product's tiles only (cost order), against GSLM_TILE_ORDER=flat: mv_ab and
# lm_phases alternated; the forward is unaffected (length order stays frame-wide)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05am
mkdir -p $O
for r in 1 2 3; do
  for m in flat xcd; do
    GSLM_TILE_ORDER=$m timeout -k 10 240 python tools/mv_ab.py $m --out /tmp/ab_am > $O/mv_${m}_$r.json 2> $O/mv_${m}_$r.err || { tail -5 $O/mv_${m}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/mv_${m}_$r.json').read().strip().splitlines()[-1]);print('$m $r', {k:round(v,4) for k,v in d.items() if k in ('cg_iter_ms','render_matvec_ms','render_matvec_loop_ms','jv_ms','forward_ms')})"
  done
done
python tools/mv_ab.py --compare /tmp/ab_am flat xcd
for m in flat xcd flat xcd; do
  GSLM_TILE_ORDER=$m timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_$m.json 2> $O/lm_$m.err || { tail -5 $O/lm_$m.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/lm_$m.json').read().strip().splitlines()[-1]);print('lm $m', d['untimed_ms'], [t['line_search_ms'] for t in d['timed']])"
done
