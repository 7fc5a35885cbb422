"""Print the interleaved A/B bench values of tools/ab_lib.sh: python tools/ab_show.py TAG"""
import json
import sys

tag = sys.argv[1]
for side in "AB":
    vals = []
    for i in (1, 2, 3):
        try:
            vals.append(json.loads(open(f"gpurun_out/{tag}_{side}{i}.json").readline())["value"])
        except Exception:                                  # a run that did not finish
            pass
    print(side, vals, f"mean {sum(vals) / max(len(vals), 1):.2f}")
