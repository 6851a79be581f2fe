#!/usr/bin/env python3
"""Host-env overlap evidence from a rocprofv3 --kernel-trace --memory-copy-trace csv run.

Classifies dispatches by thread: the rollout thread launches the sampling kernels
(mlp_forward CAT/GAUSS sample) and its H2D/D2H copies, the main thread the learner kernels.
Reports, per side, busy time and how much of the rollout side's GPU activity overlaps the
learner's kernels in wall time (the lag-1 pipeline of runtime/host_trainer.py).

    python tools/overlap_summary.py gpurun_out/prof_host/run
"""
import csv
import sys


def intervals(rows):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)


def union(iv):
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(prefix):
    ks = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
    try:
        cs = list(csv.DictReader(open(prefix + "_memory_copy_trace.csv")))
    except FileNotFoundError:
        cs = []
    learner_threads = {}
    for r in ks:
        n = r["Kernel_Name"]
        if "value_grad" in n or "mlp_grad" in n or "adam" in n:
            learner_threads[r["Thread_Id"]] = learner_threads.get(r["Thread_Id"], 0) + 1
    main_tid = max(learner_threads, key=learner_threads.get) if learner_threads else None
    learn = [r for r in ks if r["Thread_Id"] == main_tid]
    roll = [r for r in ks if r["Thread_Id"] != main_tid] + [r for r in cs if r.get("Thread_Id") != main_tid]
    L, R = union(intervals(learn)), union(intervals(roll))
    t0 = min(x[0] for x in L + R)
    t1 = max(x[1] for x in L + R)
    busy = lambda u: sum(e - s for s, e in u)  # noqa: E731
    ov = overlap(L, R)
    print(f"window {(t1 - t0) / 1e6:.2f} ms; learner-thread kernels busy {busy(L) / 1e6:.2f} ms "
          f"({len(learn)} dispatches); rollout-thread kernels+copies busy {busy(R) / 1e6:.2f} ms "
          f"({len(roll)} ops); concurrent {ov / 1e6:.2f} ms = {100 * ov / max(busy(R), 1):.1f} % of the rollout "
          f"side's GPU time runs while learner kernels run")


if __name__ == "__main__":
    main(sys.argv[1])
