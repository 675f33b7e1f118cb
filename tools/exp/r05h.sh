# round 5: the line-search blends over groups of sets (GSLM_LOSS_SETS = 1 per set, 2, 3, 8 = all) inside lm_step,
# interleaved twice, after the line-search parity tests (every group size must give the per-set losses bitwise)
set -o pipefail
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_line_search.py -v -s --timeout 200 --timeout-method thread > $O/ls_tests.log 2>&1 \
  || { tail -20 $O/ls_tests.log; exit 1; }
tail -2 $O/ls_tests.log
for r in 1 2; do
  for k in 1 2 3 8; do
    GSLM_LOSS_SETS=$k timeout -k 10 300 python -u tools/exp/lm_phases.py --reps 3 > $O/lm_k${k}_r$r.json 2> $O/lm_k${k}_r$r.err \
      || { echo "lm_phases k=$k failed"; tail -5 $O/lm_k${k}_r$r.err; exit 1; }
    echo "k=$k r=$r $(tail -c 400 $O/lm_k${k}_r$r.json)"
  done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
tail -c 3000 $O/bench.json
