"""Summarise rocprofv3 --pmc counter_collection.csv files: per kernel name, mean of each counter per dispatch."""
import csv
import sys
from collections import defaultdict


def main(paths, filt=None):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"]
                if filt and filt not in k:
                    continue
                acc[k[:90]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")


if __name__ == "__main__":
    args = sys.argv[1:]
    filt = None
    if args and args[0].startswith("--filter="):
        filt = args[0].split("=", 1)[1]
        args = args[1:]
    main(args, filt)
