# round 5: bench.py with the multi-stream raster throughput field (raster_streams)
set -o pipefail
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err \
  || { tail -20 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/r05o/bench.json").read().strip().splitlines()[-1])
print(d["value"], d["raster_mpix_s"], d["forward_ms_per_view"], d["raster_streams"], d["lm_step"]["ms"])
PY
