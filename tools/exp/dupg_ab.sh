# union duplicate block size: 128 (build_base) against 64 Gaussians per block (build_g64): union stages and the 50-view
# six points (union vs exact losses compared)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-dupg_ab}
mkdir -p $O
for L in build_base build_g64 build_base build_g64; do
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 python -u tools/exp/union_kernels.py > $O/uk_$L.json 2> $O/uk_$L.err || { echo "uk $L failed"; tail -5 $O/uk_$L.err; exit 1; }
  echo $L $(cat $O/uk_$L.json)
done
GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/build_g64/libgslm.so timeout -k 10 300 python -u tools/exp/ls_union.py --reps 2 --mode union > $O/ls_g64.json 2> $O/ls.err || { echo "ls failed"; tail -5 $O/ls.err; exit 1; }
cat $O/ls_g64.json
