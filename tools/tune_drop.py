#!/usr/bin/env python
"""Copy a committed tile-choice cache (profiles/tune_*.json) without the keys that contain any
of the given substrings, so that ``bench.py --tune-cache <out> --save-tune <new>`` re-tunes
exactly those launch shapes (e.g. after a new tile family became a candidate for them) and
keeps every other committed choice.

    python tools/tune_drop.py profiles/tune_fwd_bf16_b8_256.json gpurun_out/in.json 1/0/5/2/
"""
import json
import sys


def main():
    src, dst, *pats = sys.argv[1:]
    with open(src) as fh:
        d = json.load(fh)
    keep = {k: v for k, v in d.items() if not any(p in k for p in pats)}
    print(f"{src}: dropped {len(d) - len(keep)} of {len(d)} keys ({', '.join(pats)})")
    with open(dst, "w") as fh:
        json.dump(keep, fh, indent=0)


if __name__ == "__main__":
    main()
