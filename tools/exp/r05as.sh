# round 5: the round-4 final library (9bda87f) against the final round-5 library on one box -- tangent / matvec / gather
# stages and the CG iteration at 1M (projected layout) and at 5M in the full SH-rest layout (configs[4]'s per-view
# kernels), to see whether configs[4]'s 0.58 -> 0.75 ms tangent stage is a regression or box-to-box
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05as
mkdir -p $O
MVAB_ARGS="" bash tools/ab_run.sh r05as_1m build_r04 build build_r04 build > $O/ab_1m.txt 2>&1 || { tail -20 $O/ab_1m.txt; exit 1; }
MVAB_ARGS="--P 5000000 --full --reps 10" bash tools/ab_run.sh r05as_5m build_r04 build build_r04 build > $O/ab_5m.txt 2>&1 || { tail -20 $O/ab_5m.txt; exit 1; }
for d in r05as_1m r05as_5m; do
  for f in gpurun_out/$d/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$d', '$f'.split('/')[-1], {k:round(v,4) for k,v in d.items() if k in ('tangent_ms','render_matvec_ms','gather_ms','cg_iter_ms')})"; done
done
