# round 6 call ah: the drop-in backward's visited-row flags instead of the N x 48 B row fill (working tree -> build_rf)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_rf/libgslm.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_raster.py tests/test_gpu_edge.py tests/test_gpu_fullsize.py tests/test_gpu_dropin_memo.py tests/test_gpu_dropin_branches.py tests/test_gpu_batch_render.py tests/test_gpu_fullsize_props.py > gpurun_out/r06ah_tests.log 2>&1 || { tail -30 gpurun_out/r06ah_tests.log; exit 1; }
tail -1 gpurun_out/r06ah_tests.log
mkdir -p gpurun_out/r06ah
for L in build_head build_rf build_head build_rf; do
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 python tools/exp/dropin_breakdown.py --reps 11 > gpurun_out/r06ah/$L.$RANDOM.json 2> gpurun_out/r06ah/$L.err || { tail -5 gpurun_out/r06ah/$L.err; exit 1; }
done
for f in gpurun_out/r06ah/*.json; do echo "$f $(python3 -c "import json; d=json.load(open('$f')); print({k: round(d[k], 4) for k in d if k in ('matvec','matvec_T','forward')})")"; done
for L in build_head build_rf; do
  (cd /tmp && GSLM_ABI_ANY=1 GSLM_LIB=$GRAFT_REPO_ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/r06ah/prof_$L -o run -- python3 $GRAFT_REPO_ROOT/tools/exp/dropin_breakdown.py --reps 5 > /dev/null 2>&1) || exit 1
done
for L in build_head build_rf; do echo "== $L"; python3 -c "
import csv,glob
f=glob.glob('gpurun_out/r06ah/prof_$L/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    n=r['Name']
    if 'render_bwd' in n or 'preprocess_bwd' in n or 'fill' in n.lower(): print(n[:60], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"; done
