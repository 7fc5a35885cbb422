"""Kernel statistics from a rocprofv3 sqlite results database (the default output format of
`rocprofv3 --kernel-trace`): per kernel name, dispatches, total / average duration, share.

  python tools/prof_db_stats.py gpurun_out/prof_c3/c3_results.db [--steps N] [--top 40]

--step-marker NAME keeps one step: the dispatches between the last two of kernel NAME.
--steps N divides the totals by N (per-step figures for a bench run of N timed + warmup steps
when the trace was cut to those steps; otherwise just a scale)."""
import argparse
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--steps", type=float, default=1.0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--csv", default=None)
    ap.add_argument("--step-marker", default=None,
                    help="kernel-name substring dispatched once per step (e.g. mse_bwd_kernel): "
                         "report only the dispatches between its last two occurrences")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    where = ""
    if a.step_marker:
        st = [r[0] for r in c.execute(f"select start from kernels where {name} like ? order by start",
                                      (f"%{a.step_marker}%",))]
        assert len(st) >= 2, "marker seen fewer than twice"
        where = f"where start >= {st[-2]} and start < {st[-1]}"
        a.steps = 1.0
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start) from kernels "
                     f"{where} group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows)
    out = []
    for n, cnt, tot, avg in rows:
        out.append((n, cnt / a.steps, tot / a.steps / 1e6, avg / 1e3, 100.0 * tot / total))
    print(f"total {total / a.steps / 1e6:.3f} ms per step over {sum(r[1] for r in rows) / a.steps:.0f} "
          f"dispatches")
    for n, cnt, ms, us, pct in out[:a.top]:
        print(f"{ms:8.3f} ms {pct:5.1f}% n={cnt:7.1f} avg {us:8.2f} us  {n[:110]}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("name,dispatches_per_step,ms_per_step,avg_us,pct\n")
            for n, cnt, ms, us, pct in out:
                f.write(f'"{n}",{cnt:.2f},{ms:.4f},{us:.3f},{pct:.2f}\n')


if __name__ == "__main__":
    main()
