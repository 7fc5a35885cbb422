"""Per-kernel PMC counter averages from a rocprofv3 --pmc sqlite results database.

  python tools/pmc_db.py gpurun_out/pmc/x_results.db [--match wgrad_s2]
"""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(counters_collection)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    cname = "counter_name" if "counter_name" in cols else "counter"
    val = "value" if "value" in cols else "counter_value"
    rows = c.execute(f"select {name}, {cname}, count(*), avg({val}) from counters_collection "
                     f"where {name} like ? group by {name}, {cname}",
                     (f"%{a.match}%",)).fetchall()
    cur = None
    for n, cn, cnt, v in sorted(rows):
        if n != cur:
            print(n[:120])
            cur = n
        print(f"   {cn:32s} n={cnt:5d} avg {v:16.1f}")


if __name__ == "__main__":
    main()
