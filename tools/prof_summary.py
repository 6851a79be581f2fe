#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (or kernel_stats.csv) per kernel."""
import csv
import sqlite3
import sys
import re


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:90]


def main_csv(path):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'total ms':>9s} {'calls':>6s} {'avg us':>9s} {'pct':>5s}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t, n = float(r["TotalDurationNs"]), int(r["Calls"])
        print(f"{t / 1e6:9.2f} {n:6d} {t / n / 1e3:9.1f} {100 * t / tot:5.1f}  {r['Name'][:100]}")
    print(f"total GPU kernel time {tot / 1e6:.2f} ms")


def main(path):
    if path.endswith(".csv"):
        return main_csv(path)
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
    rows = c.execute(f"select {name_col}, start, end from kernels").fetchall()
    agg = {}
    for n, s, e in rows:
        k = short(n)
        a = agg.setdefault(k, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    print(f"{'kernel':90s} {'calls':>7s} {'total_us':>12s} {'avg_us':>10s} {'pct':>6s}")
    for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{k:90s} {n:7d} {t:12.1f} {t / n:10.2f} {100 * t / tot:6.2f}")
    print(f"total kernel time {tot / 1e3:.2f} ms over {sum(v[0] for v in agg.values())} dispatches")


if __name__ == "__main__":
    main(sys.argv[1])
