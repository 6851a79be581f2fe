"""gloo P2P on device tensors is fenced (the one-GPU rehearsal of the multi-rank path).

gloo moves a device tensor's bytes from host threads, outside stream order, so a send posted
right after the kernels that write its buffer can carry stale bytes (``tools/probes/
gloo_device_p2p_probe.py --via dist``).  ``Comm.gather_to`` and the actor-learner P2P sites
synchronise the stream first for non-RCCL backends; here two gloo ranks share cuda:0 and every
round's buffer must arrive whole.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_comm_gather_to_over_gloo_waits_for_the_writing_kernels(cuda):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "tools/probes/gloo_device_p2p_probe.py",
           "--via", "comm", "--fence", "0", "--rounds", "12"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", PYTHONPATH=REPO)
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(rec) == 1, r.stdout
    assert rec[0]["stale_or_torn_rounds"] == 0, rec[0]
