# round 6 call l: the evidence run on the final tree -- the whole GPU suite (with the parity-margin log) and the bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export GSLM_MARGINS=gpurun_out/r06l/parity_margins.jsonl
TAG=r06l TEST_TIMEOUT=900 BENCH_TIMEOUT=420 bash tools/gpu_run.sh
