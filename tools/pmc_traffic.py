"""HBM traffic per dispatch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over
tools/graph_trace.py (forward graph replays delimited by spin kernels).

FETCH_SIZE and WRITE_SIZE are KiB per dispatch.  Per /opt/skills/guides/MI355X_MICROARCH.md
(HBM section), on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads,
so it is doubled; WRITE_SIZE is taken as is.  Only dispatches inside the replay window (after
the first spin kernel) are counted.  Output: JSON {short kernel name: {...}} keyed like
bench.py's roofline kernel names.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv OUT.json [BATCH SIZE]
"""
import csv
import json
import sys
from collections import defaultdict


def short_name(k):
    """'void rgbac::conv_kernel<rgbac::bf16_t, 64, 64, 2, 2, 3>(rgbac::ConvArgsDev)' ->
    'conv_kernel<bf16_t, 64, 64, 2, 2, 3>' (the names bench.py's launch profiler uses)."""
    return k.replace("void ", "").replace("rgbac::", "").split("(")[0].strip()


def per_dispatch(path, counter):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            rows.append((int(r["Dispatch_Id"]), r["Kernel_Name"], float(r["Counter_Value"])))
    rows.sort()
    spins = [i for i, r in enumerate(rows) if "sleep" in r[1].lower() or "spin" in r[1].lower()]
    if spins:
        rows = rows[spins[0] + 1:spins[-1]]
    acc = defaultdict(lambda: [0, 0.0])
    for _, k, v in rows:
        if "sleep" in k.lower() or "spin" in k.lower():
            continue
        a = acc[short_name(k)]
        a[0] += 1
        a[1] += v
    return acc


def main(fetch_csv, write_csv, out, batch=8, size=256):
    f = per_dispatch(fetch_csv, "FETCH_SIZE")
    w = per_dispatch(write_csv, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        nf, sf = f.get(k, [0, 0.0])
        nw, sw = w.get(k, [0, 0.0])
        fb = 2.0 * sf * 1024 / max(nf, 1)
        wb = sw * 1024 / max(nw, 1)
        res[k] = {"dispatches_fetch_pass": nf, "dispatches_write_pass": nw,
                  "fetch_bytes_per_dispatch": round(fb), "write_bytes_per_dispatch": round(wb),
                  "hbm_bytes_per_dispatch": round(fb + wb)}
    with open(out, "w") as fh:
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over "
                             "tools/graph_trace.py forward graph replays; FETCH_SIZE x2 (gfx950)",
                   "config": {"batch": int(batch), "size": int(size), "dtype": "bf16"},
                   "kernels": res}, fh, indent=1)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]["hbm_bytes_per_dispatch"]):
        print(f"{v['hbm_bytes_per_dispatch'] / 1e6:9.2f} MB/dispatch  {k}")


if __name__ == "__main__":
    main(*sys.argv[1:6])
