# configs[4] per-rank emulation: 5M Gaussians, 32 4K views over n = 8, 4, 2 ranks, SH-rest coordinates and the full
# layout; then the whole batch on one GPU (bench.py headline only: the full LM step over 32 4K training views does not
# fit one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04g}
mkdir -p $O
for n in ${NS-8 4 2}; do
  for lay in coords full; do
    timeout -k 10 300 env GSLM_SHARD_REST=$lay python -u tools/exp/rank_emulate.py --P 5000000 --W 3840 --H 2160 --per $((32 / n)) --ranks $n --steps 5 --no-n1 > $O/c4_n${n}_$lay.json 2> $O/c4_n${n}_$lay.err || { echo "n=$n $lay failed"; tail -20 $O/c4_n${n}_$lay.err; exit 1; }
    cat $O/c4_n${n}_$lay.json
  done
done
timeout -k 10 400 python -u bench.py --P 5000000 --width 3840 --height 2160 --views-per-gpu 32 --steps 3 --warmup 1 --no-cpu-baseline --no-side > $O/bench_c4_1gpu.json 2> $O/bench_c4_1gpu.err || { echo "bench c4 failed"; tail -20 $O/bench_c4_1gpu.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_c4_1gpu.json')); print({k: d[k] for k in ('value', 'ms_per_step')})"
