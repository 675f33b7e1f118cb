# round 5: (1) the reworked parity bounds against the round-4 log2e perturbation (conic pre-scaled by log2 e in the
# render records: one extra rounding in every exponent); (2) A/B of the kept tree (k_render_matvec at 47 VGPRs under
# __launch_bounds__(256, 8)) against the tile-cost-order build (56 VGPRs); (3) the split profile of k_render_matvec:
# kernel trace + two SQ counter passes over tools/exp/split_passes.py
set -o pipefail
O=gpurun_out/r05d
mkdir -p $O
ROOT=$PWD
GSLM_LIB=$ROOT/gaussian-splatting-lm_amd/build_l2e/libgslm.so GSLM_MARGINS=$ROOT/$O/l2e_margins.jsonl \
  timeout -k 10 400 python -u -m pytest tests/test_gpu_drift.py tests/test_gpu_lm.py tests/test_gpu_fullsize.py -m gpu -v -s \
  -k "whole_frame_100k or drift or cgls or recursions or loss_rhs or bench_size" --timeout 300 --timeout-method thread \
  > $O/l2e_tests.log 2>&1
rc=$?
tail -3 $O/l2e_tests.log; grep -E "^FAILED" $O/l2e_tests.log | head
case $rc in 0|1) ;; *) echo "l2e run rc=$rc: stopping"; exit $rc;; esac
MVAB_ARGS="--reps 40" bash tools/ab_run.sh r05d_ab build_order build build_order build || exit 1
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$O/trace -o run -- \
   python3 $ROOT/tools/exp/split_passes.py --reps 20 --out $ROOT/$O/split.json > $ROOT/$O/trace.log 2>&1) || { echo trace failed; tail -5 $O/trace.log; exit 1; }
RE='k_render_matvec|k_render_jv_wave|k_render_bwd'
pmc() { local name=$1; shift
  (cd /tmp && timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "$RE" -f csv -d $ROOT/$O/$name -o run \
     -- python3 $ROOT/tools/exp/split_passes.py --reps 5 > $ROOT/$O/$name.log 2>&1); }
pmc p1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
&& pmc p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD \
&& python tools/sq_summary.py $O > $O/sq.txt; echo sq rc=$?
cat $O/split.json
