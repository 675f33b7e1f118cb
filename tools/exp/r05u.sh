# round 5: the multi-stream raster throughput at 2 / 4 / 8 / 12 renders in flight (bench.py's raster_streams)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05u
mkdir -p $O
for S in 4 8 12 2; do
  GSLM_RASTER_STREAMS=$S timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_s$S.json 2> $O/bench_s$S.err || { tail -5 $O/bench_s$S.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_s$S.json').read().strip().splitlines()[-1]);print($S, d['raster_streams'], d.get('raster',{}).get('mpix_s') if isinstance(d.get('raster'),dict) else d.get('raster_mpix_s'))"
done
