# round 6 call m: the evidence profiles on the final tree -- rocprofv3 kernel stats (with and without the side
# measurements), FETCH_SIZE / WRITE_SIZE passes, the per-launch PMC summary; then configs[4] whole on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_profile.sh r06m notests --no-cpu-baseline || exit 1
timeout -k 10 600 python -u bench.py --P 5000000 --width 3840 --height 2160 --views-per-gpu 32 --no-side --steps 5 --warmup 2 \
  > gpurun_out/r06m/bench_configs4_1gpu.json 2> gpurun_out/r06m/bench_configs4_1gpu.err || { tail -20 gpurun_out/r06m/bench_configs4_1gpu.err; exit 1; }
cat gpurun_out/r06m/bench_configs4_1gpu.json
