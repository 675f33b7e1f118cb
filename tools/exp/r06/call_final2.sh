# round 6 final evidence after the key-range depth sort: the whole GPU suite (parity margins logged) and the bench line, then the
# rocprofv3 kernel statistics and FETCH_SIZE / WRITE_SIZE passes (tools/gpu_profile.sh), each step time-limited
set -o pipefail
cd $GRAFT_REPO_ROOT
export GSLM_MARGINS=gpurun_out/r06final2/parity_margins.jsonl
TAG=r06final2 TEST_TIMEOUT=900 BENCH_TIMEOUT=420 bash tools/gpu_run.sh || exit 1
bash tools/gpu_profile.sh r06final2_prof notests --no-cpu-baseline || exit 1
