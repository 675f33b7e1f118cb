# round 5: the LM tile passes as independent waves (vjp_wave_lm: quadrant rows, no block barrier) -- the whole GPU
# suite, then bench.py and a kernel-trace profile of it
set -o pipefail
O=gpurun_out/r05i
mkdir -p $O
ROOT=$PWD
export GSLM_MARGINS=$ROOT/$O/parity_margins.jsonl
rm -f $GSLM_MARGINS
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log; grep -E "^FAILED" $O/gpu_tests.log | head -20
case $rc in 0|1) ;; *) echo "test rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
head -c 1500 $O/bench.json; echo
python - <<'PY'
import json
b = json.loads(open("gpurun_out/r05i/bench.json").read().strip().splitlines()[-1])
print("stage_ms", b.get("stage_ms"), "lm_step", b.get("lm_step", {}).get("ms"), "ssim", b.get("ssim_cg"))
PY
