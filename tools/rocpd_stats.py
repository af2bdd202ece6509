"""Per-kernel summary of a rocprofv3 rocpd database (the default output of
ROCm 7's rocprofv3): calls, total and average duration, share.

    python tools/rocpd_stats.py gpurun_out/prof/x_results.db [--per N] [--csv out.csv]
--per N divides call counts by N (e.g. ticks) to give kernels per unit.
"""
import argparse
import csv
import re
import sqlite3


def short(name, n=90):
    s = re.sub(r"\(.*$", "", name)
    s = re.sub(r"^void ", "", s)
    return s if len(s) <= n else s[:n - 3] + "..."


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("--per", type=float, default=0)
    p.add_argument("--csv", default=None)
    p.add_argument("--top", type=int, default=40)
    a = p.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, count(*), sum(duration), avg(duration) from kernels group by name "
                     "order by sum(duration) desc").fetchall()
    tot = sum(r[2] for r in rows)
    calls = sum(r[1] for r in rows)
    print(f"{len(rows)} kernels, {calls} dispatches, {tot / 1e6:.3f} ms total")
    for name, n, s, avg in rows[:a.top]:
        per = f" {n / a.per:6.2f}/unit" if a.per else ""
        print(f"{s / tot * 100:5.1f}% {n:7d}{per} avg {avg / 1e3:8.2f} us  {short(name)}")
    if a.per:
        print(f"per unit: {calls / a.per:.1f} dispatches, {tot / a.per / 1e3:.1f} us of kernel time")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
            for name, n, s, avg in rows:
                w.writerow([name, n, s, avg, s / tot * 100])


if __name__ == "__main__":
    main()
