# round 6 call n: the CG loop's two dot finalisation launches priced (timing-only build without them)
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06n build build_nofinal build build_nofinal > gpurun_out/r06n.log 2>&1 || { tail -20 gpurun_out/r06n.log; exit 1; }
grep -v "^\[" gpurun_out/r06n.log | tail -12
