set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04c
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -k "line_search or lm_step or gshard or rccl or dist or configs34 or rest_coords" > gpurun_out/r04c/gpu_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r04c/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r04c/gpu_tests.log
timeout -k 10 300 python -u tools/exp/ls_union.py --reps 3 > gpurun_out/r04c/ls.json 2> gpurun_out/r04c/ls.err || { echo "ls failed"; tail -20 gpurun_out/r04c/ls.err; exit 1; }
cat gpurun_out/r04c/ls.json
