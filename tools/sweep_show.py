"""Values of a tools/r03_sweep.sh run: python tools/sweep_show.py TAG"""
import glob
import json
import os
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}_*.json"), key=os.path.getmtime):
    try:
        d = json.loads(open(f).readline())
        print(f"{os.path.basename(f):24s} {d['value']:8.2f} {d['ms_per_step']:.3f}")
    except Exception as e:                                 # a run that did not finish
        print(f, e)
