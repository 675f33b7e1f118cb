"""Per-kernel averages of the SQ / GRBM counter passes written by tools/sq_counters.sh."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(out):
    acc = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(out, "*", "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0]
                acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"  {c:24s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
