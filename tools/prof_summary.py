#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (or kernel_stats.csv) per kernel."""
import sqlite3
import sys
import re


def short(n):
    n = re.sub(r"\(.*", "", n)
    return n[:90]


def main(path):
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
