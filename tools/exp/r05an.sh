# round 5: k_render_matvec's counted HBM fetch with the XCD-aware LM tile order against the frame-wide one
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05an
mkdir -p $O
export TMPDIR=/tmp
ROOT=$PWD
for m in flat xcd; do
  (cd /tmp && GSLM_TILE_ORDER=$m timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_render_matvec -f csv -d $ROOT/$O/pmc_$m -o run \
     -- python3 $ROOT/bench.py --no-cpu-baseline --no-side --steps 10 --warmup 3 --forward-steps 2 > /dev/null 2> $ROOT/$O/pmc_$m.err) || { tail -5 $O/pmc_$m.err; exit 1; }
  python3 - <<PY
import csv,glob
v=[float(r['Counter_Value']) for f in glob.glob('$O/pmc_$m/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if 'k_render_matvec<false>' in r['Kernel_Name']]
print('$m', len(v), 'FETCH_SIZE KiB avg', sum(v)/len(v), 'x2 bytes', 2*1024*sum(v)/len(v))
PY
done
