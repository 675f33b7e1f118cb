# round 5: the J v loop's bound test against the lane's per-round bound (no scalar add per visit): GPU suite, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ar
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
bash tools/ab_run.sh r05ar build_base build build_base build build_base build > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -4 $O/ab.txt
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f'.split('/')[-1], {k:round(v,4) for k,v in d.items() if k in ('cg_iter_ms','render_matvec_ms','jv_ms')})"; done
