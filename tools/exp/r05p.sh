# round 5: k_gather_lm (projected layout) at 7 waves per SIMD (32 B of spill) against the kept 6 -- CG-loop A/B
set -o pipefail
O=gpurun_out/r05p
mkdir -p $O
ROOT=$PWD
for r in 1 2 3; do
  for L in build build_g7; do
    GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 python -u tools/mv_ab.py $L --reps 40 --out /tmp/ab \
      > $O/ab_${L}_$r.json 2> $O/ab_${L}_$r.err || { echo "mv_ab $L failed"; tail -5 $O/ab_${L}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/ab_${L}_$r.json').read().strip().splitlines()[-1]);print('$L', d['gather_ms'], d['cg_iter_ms'])"
  done
done
timeout -k 10 120 python -u tools/mv_ab.py --compare /tmp/ab build build_g7
