# configs[3] per-rank emulation (1M Gaussians, one 1080p view per rank) at n = 2, 4, 8, SH-rest coordinates, with the
# single-view N = 1 iterations beside it
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04c3}
mkdir -p $O
for n in 2 4 8; do
  extra=""; [ $n != 8 ] && extra="--no-n1"
  timeout -k 10 300 python -u tools/exp/rank_emulate.py --ranks $n --steps 20 $extra > $O/c3_n$n.json 2> $O/c3_n$n.err || { echo "n=$n failed"; tail -20 $O/c3_n$n.err; exit 1; }
  cat $O/c3_n$n.json
done
