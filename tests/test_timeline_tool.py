"""tools/timeline.py: one update's kernel timeline from a rocprofv3 kernel-trace csv."""
import csv
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, updates=4):
    cols = ["Kind", "Agent_Id", "Queue_Id", "Stream_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"]
    rows, t = [], 1_000_000
    for _ in range(updates):
        # main queue: fwd 50 us, gap 2 us, bwd 100 us, adam 10 us; side queue: wgrad 40 us beside bwd
        for q, name, dt, gap in (("1", "conv_fwd_kernel", 50_000, 0), ("1", "conv_bwd_kernel", 100_000, 2_000),
                                 ("1", "adam_clip4_kernel", 10_000, 0)):
            t += gap
            rows.append({"Kind": "KERNEL_DISPATCH", "Agent_Id": "1", "Queue_Id": q, "Stream_Id": "0",
                         "Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dt})
            if name == "conv_bwd_kernel":
                rows.append({"Kind": "KERNEL_DISPATCH", "Agent_Id": "1", "Queue_Id": "2", "Stream_Id": "1",
                             "Kernel_Name": "wgrad_kernel", "Start_Timestamp": t + 5_000, "End_Timestamp": t + 45_000})
            t += dt
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        w.writerows(rows)


def test_timeline_reports_one_update_with_gaps_and_queue_busy(tmp_path):
    _trace(tmp_path / "run_kernel_trace.csv")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "timeline.py"), str(tmp_path) + "/"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout
    assert "update of 4 kernels, 162.0 us" in out  # fwd + 2 us gap + bwd + adam
    assert "conv_bwd_kernel" in out and "wgrad_kernel" in out
    gap_line = [ln for ln in out.splitlines() if "conv_bwd_kernel" in ln][0]
    assert gap_line.split()[2] == "2.0"  # the main queue's idle gap before the backward
    assert "stream 1: busy 160.0 us of 162.0" in out and "stream 2: busy 40.0 us" in out
