set -o pipefail
O=gpurun_out/r03s2_devab
mkdir -p $O
timeout -k 10 400 python -u tools/exp/val_time.py --streams 8 --readback --reps 3 > $O/val_time.json 2> $O/val_time.err || { tail -20 $O/val_time.err; exit 1; }
cat $O/val_time.json
