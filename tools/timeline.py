#!/usr/bin/env python3
"""One update's kernel timeline from a rocprofv3 --kernel-trace csv run.

Splits the trace into updates at each ``--marker`` kernel (default: the Adam launch that ends
a Pong A2C update), takes the median-length update among the last ``--updates``, and prints
every kernel of it: start offset, duration, stream, and the gap on its stream since the
previous kernel there; then per-stream busy time and the critical (main) stream's idle time.

    python tools/timeline.py gpurun_out/tl2048/run
"""
import argparse
import csv
import glob
import os
import statistics


def load(prefix):
    paths = glob.glob(prefix + "*kernel_trace.csv") or glob.glob(os.path.join(prefix, "**", "*kernel_trace.csv"),
                                                                  recursive=True)
    if not paths:
        raise SystemExit(f"no kernel_trace.csv under {prefix}")
    rows = []
    for p in paths:
        with open(p) as f:
            rows += list(csv.DictReader(f))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["q"] = r.get("Queue_Id") or r.get("Stream_Id")
    return sorted(rows, key=lambda r: r["s"])


def short(name, n=64):
    name = name.replace("void ", "").replace("rrl::", "")
    return name[:n]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--marker", default="adam_clip4_kernel")
    ap.add_argument("--updates", type=int, default=6)
    a = ap.parse_args()
    rows = load(a.prefix)
    ends = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(ends) < 3:
        raise SystemExit(f"fewer than 3 '{a.marker}' launches")
    spans = [(ends[k - 1] + 1, ends[k] + 1) for k in range(max(1, len(ends) - a.updates), len(ends))]
    lens = [rows[j - 1]["e"] - rows[i]["s"] for i, j in spans]
    med = sorted(zip(lens, spans))[len(lens) // 2]
    i0, i1 = med[1]
    upd = rows[i0:i1]
    t0 = upd[0]["s"]
    print(f"update of {len(upd)} kernels, {med[0] / 1e3:.1f} us first start -> last end "
          f"(median of the last {len(lens)}: {statistics.median(lens) / 1e3:.1f} us)")
    last_end = {}
    busy = {}
    print(f"{'start':>8} {'dur':>7} {'gap':>6} {'q':>3}  kernel")
    for r in upd:
        q = r["q"]
        gap = (r["s"] - last_end[q]) / 1e3 if q in last_end else 0.0
        last_end[q] = max(last_end.get(q, 0), r["e"])
        busy[q] = busy.get(q, 0) + (r["e"] - r["s"])
        print(f"{(r['s'] - t0) / 1e3:8.1f} {(r['e'] - r['s']) / 1e3:7.1f} {gap:6.1f} {q:>3}  {short(r['Kernel_Name'])}")
    span = med[0]
    for q, b in sorted(busy.items(), key=lambda kv: -kv[1]):
        print(f"stream {q}: busy {b / 1e3:.1f} us of {span / 1e3:.1f} ({100 * b / span:.1f} %)")


if __name__ == "__main__":
    main()
