# round 6 call s: the final tree's evidence -- the whole GPU suite and the bench line (as call_l.sh), then the kernel
# statistics of configs[4] whole on one GPU (the LM row map's scans at 59M pairs per 4K view: ADVICE r05)
set -o pipefail
cd $GRAFT_REPO_ROOT
export GSLM_MARGINS=gpurun_out/r06s/parity_margins.jsonl
TAG=r06s TEST_TIMEOUT=900 BENCH_TIMEOUT=420 bash tools/gpu_run.sh || exit 1
ROOT=$(pwd)
(cd /tmp && TMPDIR=/tmp timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/gpurun_out/r06s/stats_c4" -o run \
   -- python3 "$ROOT/bench.py" --P 5000000 --width 3840 --height 2160 --views-per-gpu 32 --no-side --steps 3 --warmup 1 \
   > "$ROOT/gpurun_out/r06s/bench_c4_prof.json" 2> "$ROOT/gpurun_out/r06s/bench_c4_prof.err") || { tail -20 gpurun_out/r06s/bench_c4_prof.err; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r06s/stats_c4/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("k_row_flags", "k_row_final", "k_tile_neff", "k_scan", "k_render_matvec", "k_gather_lm")):
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"]) / 1e3:9.1f} us')
PY
