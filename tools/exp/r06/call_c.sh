# round 6 call c: the forward with the 3-pass 11-bit depth sort (build) against the 4-pass 8-bit one (build_old,
# c5ecb02): mv_ab alternated, and each build's last-forward kernel timeline; the barrier-free VJP timing variant
set -o pipefail
cd $GRAFT_REPO_ROOT
MVAB_ARGS="--reps 30" timeout -k 10 600 bash tools/ab_run.sh r06c_ab build_old build build_old build build_nobar > gpurun_out/r06c_ab.log 2>&1 || { tail -20 gpurun_out/r06c_ab.log; exit 1; }
grep -v "^\[" gpurun_out/r06c_ab.log | grep tag
bash tools/prof_forward.sh build_old > gpurun_out/r06c_prof_old.txt 2>&1 || { tail gpurun_out/r06c_prof_old.txt; exit 1; }
bash tools/prof_forward.sh build > gpurun_out/r06c_prof_new.txt 2>&1 || { tail gpurun_out/r06c_prof_new.txt; exit 1; }
cat gpurun_out/r06c_prof_old.txt gpurun_out/r06c_prof_new.txt
