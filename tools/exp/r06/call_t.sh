# round 6 call t: the multi-rank rehearsals on the final tree (gloo 2 ranks on one GPU through bench.py --gpus 2; the
# one-rank RCCL Gaussian-sharded bench, both communicators) -- the N > 1 path the driver's 8-GPU run takes
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06t
mkdir -p $O
GSLM_BENCH_DIST=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "gloo2 failed: $?"; tail -30 $O/bench_gloo2.err; exit 1; }
head -c 300 $O/bench_gloo2.json; echo
GSLM_FORCE_COLLECTIVES=1 GSLM_BENCH_EXCHANGE=gaussian timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-side \
  > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { echo "rccl1 failed: $?"; tail -30 $O/bench_rccl1.err; exit 1; }
head -c 300 $O/bench_rccl1.json; echo
GSLM_COMM=native GSLM_FORCE_COLLECTIVES=1 GSLM_BENCH_EXCHANGE=gaussian timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-side \
  > $O/bench_rccl1_native.json 2> $O/bench_rccl1_native.err || { echo "rccl1 native failed: $?"; tail -30 $O/bench_rccl1_native.err; exit 1; }
head -c 300 $O/bench_rccl1_native.json; echo
