# round 5: bench line after moving the multi-stream raster measurement behind the roofline's kernel timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05z2
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['avg_launch_ms'], d['stage_ms'], d['raster_streams']['ms_per_render'], d['lm_step']['ms'])"
