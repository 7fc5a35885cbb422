"""MFMA utilisation per kernel from one rocprofv3 --pmc pass over tools/graph_trace.py
(SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE).

Per /opt/skills/guides/MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles (32 per
32x32x16 bf16 MFMA = 1024 FLOP per busy cycle per SIMD at the dense rate), summed over the
chip; GRBM_GUI_ACTIVE is summed over the 8 XCDs.  So per dispatch

    mfma_util = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 256 CUs * 4 SIMDs)

is the fraction of the chip's MFMA issue slots that were busy while the dispatch ran (it reads
low on dispatches shorter than ~0.3 ms, whose GRBM window includes launch ramp-up).  Only
dispatches inside the replay window (between the first and last spin kernels) are counted.

  python tools/pmc_mfma.py COUNTERS.csv OUT.json
"""
import csv
import json
import sys
from collections import defaultdict

from pmc_traffic import short_name


def main(path, out):
    disp = defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        names[d] = r["Kernel_Name"]
    ids = sorted(disp)
    spins = [i for i in ids if "sleep" in names[i].lower() or "spin" in names[i].lower()]
    if spins:
        ids = [i for i in ids if spins[0] < i < spins[-1]]
    acc = defaultdict(lambda: defaultdict(float))
    for i in ids:
        k = short_name(names[i])
        if "sleep" in k.lower():
            continue
        a = acc[k]
        a["n"] += 1
        for c, v in disp[i].items():
            a[c] += v
    res = {}
    tot_busy = tot_slots = 0.0
    for k, a in acc.items():
        n = a["n"]
        busy = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        grbm = a.get("GRBM_GUI_ACTIVE", 0.0)
        slots = grbm / 8 * 256 * 4
        tot_busy += busy
        tot_slots += slots
        res[k] = {"dispatches": int(n),
                  "mfma_busy_cycles_per_dispatch": busy / n,
                  "grbm_gui_active_per_dispatch": grbm / n,
                  "sq_busy_cu_cycles_per_dispatch": a.get("SQ_BUSY_CU_CYCLES", 0.0) / n,
                  "waves_per_dispatch": a.get("SQ_WAVES", 0.0) / n,
                  "mfma_util": busy / slots if slots else None}
    res["_all_dispatches"] = {"mfma_util": tot_busy / tot_slots if tot_slots else None}
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -(kv[1].get("mfma_busy_cycles_per_dispatch", 0)
                                                     * kv[1].get("dispatches", 0))):
        u = v["mfma_util"]
        print(f"{(u or 0) * 100:6.1f}%  n={v.get('dispatches', '-')!s:4s} {k}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
