# round 5 final: SQ / GRBM counters of k_render_matvec (bench.py --no-side), then configs[4] on one GPU (5M Gaussians,
# 32 4K views: the forward rate BASELINE.md quotes and the CG iteration over the batch)
set -o pipefail
O=gpurun_out/r05n
mkdir -p $O
bash tools/sq_counters.sh r05n/sq k_render_matvec > $O/sq_summary.txt 2> $O/sq.err || { echo "sq failed"; tail -5 $O/sq.err; exit 1; }
cat $O/sq_summary.txt
rm -rf $O/sq/p1/*trace* $O/sq/p2/*trace* 2>/dev/null
timeout -k 10 600 python -u bench.py --P 5000000 --width 3840 --height 2160 --views-per-gpu 32 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-side > $O/bench_c4_1gpu.json 2> $O/bench_c4_1gpu.err || { echo "bench c4 failed"; tail -20 $O/bench_c4_1gpu.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4_1gpu.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','raster_mpix_s','forward_ms_per_view','num_rendered')})"
