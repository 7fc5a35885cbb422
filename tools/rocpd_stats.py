"""Per-kernel duration stats from a rocprofv3 rocpd database (the default output format of
ROCm 7.x): python tools/rocpd_stats.py <results.db> [--top N] [--grep STR]"""
import argparse
import glob
import sqlite3


def stats(db):
    c = sqlite3.connect(db)
    tabs = [r[0] for r in c.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in c.execute(f"pragma table_info({ks})")]
    name_col = "display_name" if "display_name" in cols else "kernel_name"
    rows = c.execute(f"select s.{name_col}, d.end - d.start from {kd} d join {ks} s "
                     f"on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, dur in rows:
        a = agg.setdefault(name, [])
        a.append(dur)
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--grep", default=None)
    args = ap.parse_args()
    dbs = glob.glob(args.db)
    agg = {}
    for db in dbs:
        for k, v in stats(db).items():
            agg.setdefault(k, []).extend(v)
    tot = sum(sum(v) for v in agg.values())
    print(f"{'calls':>7} {'avg us':>10} {'min us':>10} {'total us':>12} {'%':>6}  name")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:args.top]:
        if args.grep and args.grep not in k:
            continue
        print(f"{len(v):7d} {sum(v) / len(v) / 1e3:10.2f} {min(v) / 1e3:10.2f} "
              f"{sum(v) / 1e3:12.1f} {100.0 * sum(v) / tot:6.2f}  {k[:120]}")


if __name__ == "__main__":
    main()
