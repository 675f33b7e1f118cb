# configs[4] per-rank emulation: 5M Gaussians, 32 4K views over n = 8, 4, 2 ranks (and configs[3] at n = 8)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04g}
mkdir -p $O
for n in 8 4 2; do
  timeout -k 10 300 python -u tools/exp/rank_emulate.py --P 5000000 --W 3840 --H 2160 --per $((32 / n)) --ranks $n --steps 5 --no-n1 > $O/c4_n$n.json 2> $O/c4_n$n.err || { echo "n=$n failed"; tail -20 $O/c4_n$n.err; exit 1; }
  cat $O/c4_n$n.json
done
