"""Collective preflight: prove the multi-rank communication path in throw-away child processes
before the benchmark's ranks touch the GPU.

At world > 1 every epoch's optimiser all-reduces live inside hipGraphs (learner.py,
``Comm.graph_safe``), and the actor-learner phase uses RCCL point-to-point.  Those have only
ever run on a one-rank communicator; a node whose RCCL cannot capture (or cannot connect)
must not cost the whole scaling record.  So, on each rank, BEFORE anything initialises HIP:

1. rank 0 picks a free port and publishes it through the torchrun agent's TCP store (the
   store the launcher already runs at MASTER_ADDR:MASTER_PORT; workers are its clients);
2. every rank starts ``python -m relayrl_prototype_amd.parallel.preflight`` as a CHILD with that
   rendezvous (never an exec) and waits for it with a deadline; the child
     a. initialises the process group (RCCL / gloo),
     b. all-reduces a 70 KB fp32 buffer (the flat-gradient size of the flagship MLP),
     c. runs one point-to-point ring exchange (batch_isend_irecv, the fan-in primitive),
     d. captures one all-reduce into a CUDA/HIP graph, replays it 3 times on fresh inputs and
        compares every result BITWISE with the eager all-reduce of the same inputs,
   and prints one JSON line; a child past the deadline is killed (its process group);
3. the ranks exchange their results through the store and decide the same thing:
   ``rccl_ok`` (a+b+c on every rank) and ``graphs_ok`` (d on every rank).

The parent then runs eagerly if ``graphs_ok`` is false, and reports the failure instead of a
number if ``rccl_ok`` is false.  ``RRL_PREFLIGHT_INJECT=capture|rccl|hang`` injects a failure
(tests: the fallback paths on a one-GPU box or over gloo).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import subprocess
import sys
import time
from typing import Any, Dict, Optional

N_FLOATS = 17_920  # 70 KB of fp32: the flagship's flat gradient is ~70 KB (comm.py docstring)


def _child(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--timeout-s", type=float, default=45.0)
    a = ap.parse_args(argv)
    inject = os.environ.get("RRL_PREFLIGHT_INJECT", "")
    res: Dict[str, Any] = {"rank": a.rank, "backend": a.backend, "rccl_ok": False, "graphs_ok": False,
                           "stage": "init"}
    t0 = time.perf_counter()
    try:
        import datetime

        import torch
        import torch.distributed as dist

        if inject == "hang" and a.rank == 0:
            time.sleep(3600)
        if inject == "rccl":
            raise RuntimeError("injected RCCL failure")
        use_gpu = a.backend == "nccl"
        dev = torch.device("cuda", a.device) if use_gpu else torch.device("cpu")
        if use_gpu:
            torch.cuda.set_device(dev)
        dist.init_process_group(a.backend, init_method=f"tcp://127.0.0.1:{a.port}", rank=a.rank,
                                world_size=a.world, timeout=datetime.timedelta(seconds=a.timeout_s))
        res["init_s"] = round(time.perf_counter() - t0, 3)

        def inputs(k):
            g = torch.Generator().manual_seed(1000 * k + a.rank)
            return torch.randn(N_FLOATS, generator=g).to(dev)

        # b. eager all-reduce, checked against the sum of every rank's inputs
        res["stage"] = "all_reduce"
        x = inputs(0)
        ref = sum(torch.randn(N_FLOATS, generator=torch.Generator().manual_seed(r)) for r in range(a.world))
        dist.all_reduce(x)
        if use_gpu:
            torch.cuda.synchronize()
        if not torch.allclose(x.cpu(), ref, rtol=1e-5, atol=1e-5):
            raise RuntimeError("eager all-reduce returned a wrong sum")
        # c. point-to-point ring (send to rank + 1, receive from rank - 1)
        res["stage"] = "p2p"
        if a.world > 1:  # (a one-rank group has no peer to exchange with)
            send = torch.full((1024,), float(a.rank), device=dev)
            recv = torch.empty(1024, device=dev)
            nxt, prv = (a.rank + 1) % a.world, (a.rank - 1) % a.world
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, send, nxt),
                                             dist.P2POp(dist.irecv, recv, prv)]):
                w.wait()
            if use_gpu:
                torch.cuda.synchronize()
            if not bool((recv.cpu() == float(prv)).all()):
                raise RuntimeError("point-to-point exchange delivered wrong data")
        res["rccl_ok"] = True
        # d. one captured all-reduce, replayed 3x, bitwise against eager
        res["stage"] = "capture"
        if not use_gpu:
            res["graphs_ok"] = False
            res["graphs_note"] = "gloo collectives are host calls: nothing to capture"
        else:
            if inject == "capture":
                raise RuntimeError("injected graph-capture failure")
            static = torch.zeros(N_FLOATS, device=dev)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):  # warm-up on the capture stream (RCCL's own setup)
                dist.all_reduce(static)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                dist.all_reduce(static)
            for k in range(1, 4):
                xin = inputs(k)
                static.copy_(xin)
                g.replay()
                eager = xin.clone()
                dist.all_reduce(eager)
                torch.cuda.synchronize()
                if not torch.equal(static, eager):
                    raise RuntimeError(f"captured all-reduce replay {k} differs from eager")
            res["graphs_ok"] = True
        res["stage"] = "done"
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 -- reported to the parent
        res["error"] = f"{type(e).__name__}: {e}"[:400]
    res["seconds"] = round(time.perf_counter() - t0, 3)
    print("RRL_PREFLIGHT " + json.dumps(res), flush=True)
    return 0 if res["rccl_ok"] else 1


def _store(world: int, timeout_s: float):
    import datetime

    import torch.distributed as dist

    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() != "true":
        return None
    return dist.TCPStore(os.environ.get("MASTER_ADDR", "127.0.0.1"), int(os.environ["MASTER_PORT"]), world, False,
                         timeout=datetime.timedelta(seconds=timeout_s))


def run_preflight(backend: str, device: int, deadline_s: float = 90.0) -> Optional[Dict[str, Any]]:
    """Parent side, on every rank of a torchrun job, before any HIP call.  Returns the agreed
    ``{"rccl_ok", "graphs_ok", "per_rank", "seconds"}``, or None when there is no agent store
    to rendezvous through (not launched by torchrun)."""
    import socket

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    t0 = time.perf_counter()
    store = _store(world, deadline_s + 60)
    if store is None:
        return None
    pfx = f"rrl_preflight_{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}_"
    if rank == 0:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        store.set(pfx + "port", str(port))
    port = int(store.get(pfx + "port").decode())
    env = dict(os.environ)
    repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = repo + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT", "TORCHELASTIC_USE_AGENT_STORE"):
        env.pop(k, None)  # the child rendezvous is its own
    cmd = [sys.executable, "-m", "relayrl_prototype_amd.parallel.preflight", "--port", str(port), "--rank", str(rank),
           "--world", str(world), "--backend", backend, "--device", str(device),
           "--timeout-s", str(max(10.0, deadline_s - 15.0))]
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        out, err = p.communicate(timeout=deadline_s)
        res = None
        for line in out.splitlines():
            if line.startswith("RRL_PREFLIGHT "):
                res = json.loads(line[len("RRL_PREFLIGHT "):])
        if res is None:
            res = {"rank": rank, "rccl_ok": False, "graphs_ok": False, "stage": "child",
                   "error": f"child exited {p.returncode} without a result: {err[-300:]}"}
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.communicate()
        res = {"rank": rank, "rccl_ok": False, "graphs_ok": False, "stage": "timeout",
               "error": f"preflight child past its {deadline_s:.0f} s deadline (killed)"}
    store.set(pfx + f"res{rank}", json.dumps(res))
    per_rank = [json.loads(store.get(pfx + f"res{r}").decode()) for r in range(world)]
    # a rank whose child timed out while others finished: the peers' results say which stage hung
    return {"rccl_ok": all(r.get("rccl_ok") for r in per_rank),
            "graphs_ok": all(r.get("graphs_ok") for r in per_rank),
            "per_rank": per_rank, "seconds": round(time.perf_counter() - t0, 3), "backend": backend}


if __name__ == "__main__":
    sys.exit(_child())
