"""RCCL on the MI355X (the `nccl` backend of torch.distributed on ROCm).

A one-GPU box cannot host two RCCL ranks (RCCL refuses two ranks on one device), so the
multi-rank data plane is exercised here with a one-rank RCCL communicator: init over TCP on
127.0.0.1, all_reduce / broadcast / all_gather on HBM tensors, and the hipGraph capture of an
all_reduce that a captured multi-rank value loop would rely on (tools/rccl_probe.py, run in a
child process so the process group does not leak into the other tests).  The 2..8-rank
paths are covered by the gloo CPU tests (tests/test_distributed.py) and
tests/test_bench_gpu.py's two-rank RCCL test where two GPUs exist.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_one_rank_collectives_and_graph_capture(cuda):  # noqa: ARG001 (GPU fixture)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_probe.py")], env=env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["backend"] == "nccl" and out["world"] == 1
    assert out["collectives_ok"], out
    assert out["graph_capture_ok"], out
    assert out["all_reduce_69KB_us"] < 1000.0, out
