#!/bin/bash
# A/B of the Gaussian-sharded exchange's kernels for library builds (run through gpurun from the repo root):
#   bash tools/exp/gst_ab.sh <build_dir>...
# rocprofv3 kernel stats of tools/exp/gshard_time.py (one rank, 8 views) per build; prints the tangent-views,
# screen row-sum and screen-gather averages.
set -o pipefail
export TMPDIR=/tmp
for L in "$@"; do
  OUT=$GRAFT_REPO_ROOT/gpurun_out/gstab/$L; mkdir -p $OUT
  (cd /tmp && GSLM_LIB=$GRAFT_REPO_ROOT/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/exp/gshard_time.py --views 8 > $OUT/out.txt 2> $OUT/err.txt) || exit 1
  echo "== $L $(cat $OUT/out.txt)"
  grep -E "k_tangent_views|k_gather_screen|k_rowsum_screen" $(find $OUT -name "*kernel_stats.csv") | awk -F'",' '{print $1"\"", $2}' | cut -c1-150
done
