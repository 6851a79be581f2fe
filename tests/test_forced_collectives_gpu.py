"""The world > 1 optimiser path, captured into hipGraphs with its RCCL all-reduces, on one GPU.

A one-GPU box cannot host two RCCL ranks, so ``RRL_FORCE_COLLECTIVES=1`` sends a one-rank
RCCL group through the multi-rank code (``Comm.multi``: slab reduce -> ``dist.all_reduce`` ->
Adam; Pong's bucketed async all-reduces).  Captured and eager runs of that path must agree
bitwise (tools/forced_collectives_probe.py, in a child process that owns the process group).
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_forced_multi_rank_path_captured_equals_eager(cuda):  # noqa: ARG001 (GPU fixture)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "forced_collectives_probe.py"), "--check"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["multi"] and out["backend"] == "nccl" and out["graph_safe"], out
    assert out["vec_graph_replays"] >= 3 and out["vec_eager_replays"] == 0, out
    assert out["vec_pi_bitwise"] and out["vec_vf_bitwise"] and out["vec_versions_equal"], out
    assert out["pong_graphs"] >= 1 and out["pong_eager_graphs"] == 0, out
    assert out["pong_params_bitwise"], out


def test_multi_rank_engine_loop_does_not_sync_the_host_per_epoch(cuda):  # noqa: ARG001
    """with the stop agreement of a relay-attached rank 0 and log_every=0,
    the world > 1 engine loop makes no synchronising host read in steady state (the stop /
    max_seconds decision is a device flag read one epoch late), and its epoch stays within a
    few % of the world-1 graph path."""
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "forced_collectives_probe.py"), "--syncs"],
                       env=env, capture_output=True, text=True, timeout=170)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["forced_relay_sync_reads_per_epoch"] == 0, out
    assert out["forced_relay_lagged_event_waits_per_epoch"] <= 1.0, out
    assert out["relay_overhead_pct"] < 5.0, out
