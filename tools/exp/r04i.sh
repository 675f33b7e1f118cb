# union stages standalone, then the line-search tests / timing / profile / drop-in / bench (r04e.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
timeout -k 10 300 python -u tools/exp/union_kernels.py > $O/uk.json 2> $O/uk.err || { echo "uk failed"; tail -20 $O/uk.err; exit 1; }
cat $O/uk.json
bash tools/exp/r04e.sh
