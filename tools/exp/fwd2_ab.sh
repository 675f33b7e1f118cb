# A/B of the forward blend's two-visit loop: tools/mv_ab.py (forward, CG stages; products and images compared) and
# the union-list stages (slot blends), base = HEAD build, build = working tree
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-fwd2_ab}
mkdir -p $O
bash tools/ab_run.sh ${TAG:-fwd2_ab} build_base build build_base build > $O/ab.txt 2>&1 || { echo "ab failed"; tail -20 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
for L in build_base build build_base build; do
  GSLM_ABI_ANY=1 GSLM_LIB=$PWD/gaussian-splatting-lm_amd/$L/libgslm.so timeout -k 10 240 python -u tools/exp/union_kernels.py > $O/uk_$L.json 2> $O/uk_$L.err || { echo "uk $L failed"; tail -5 $O/uk_$L.err; exit 1; }
  echo $L; cat $O/uk_$L.json
done
