# round 5 final tree (final, batched final sums): GPU suite, bench line, rocprof kernel stats, FETCH/WRITE PMC, SQ counters, configs[4]
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile.sh r05aw tests || exit 1
bash tools/sq_counters.sh r05aw_sq k_render_matvec bench > gpurun_out/r05aw_sq.txt 2>&1 || { tail -5 gpurun_out/r05aw_sq.txt; exit 1; }
rm -rf gpurun_out/r05aw_sq/p1/*trace* gpurun_out/r05aw_sq/p2/*trace* 2>/dev/null
O=gpurun_out/r05aw
timeout -k 10 600 python -u bench.py --P 5000000 --width 3840 --height 2160 --views-per-gpu 32 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-side > $O/bench_c4_1gpu.json 2> $O/bench_c4_1gpu.err || { echo "bench c4 failed"; tail -20 $O/bench_c4_1gpu.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench_c4_1gpu.json').read().strip().splitlines()[-1])
print({k: d.get(k) for k in ('value','ms_per_step','raster_mpix_s','forward_ms_per_view','num_rendered')})"
