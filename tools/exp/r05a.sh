# round 5: tile schedule statistics of k_render_matvec (tools/exp/tile_sched.py) and the A/B harness's baseline
set -o pipefail
mkdir -p gpurun_out/r05a
timeout -k 10 300 python -u tools/exp/tile_sched.py --out gpurun_out/r05a/tile_sched.json > gpurun_out/r05a/tile_sched.log 2>&1
echo rc=$?
