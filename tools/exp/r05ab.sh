# round 5: the multi-rank rehearsals on one GPU after the bench.py reordering (gloo 2 ranks; one-rank RCCL exchange)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ab
mkdir -p $O
GSLM_BENCH_DIST=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline \
  > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { echo "gloo2 failed: $?"; tail -30 $O/bench_gloo2.err; exit 1; }
head -c 600 $O/bench_gloo2.json; echo
GSLM_FORCE_COLLECTIVES=1 GSLM_BENCH_EXCHANGE=gaussian timeout -k 10 600 python -u bench.py --no-cpu-baseline \
  > $O/bench_rccl1.json 2> $O/bench_rccl1.err || { echo "rccl1 failed: $?"; tail -30 $O/bench_rccl1.err; exit 1; }
head -c 600 $O/bench_rccl1.json; echo
