#!/usr/bin/env python3
"""The TrainingServer's ingest ceiling with the Python learner service in the loop.

fanin_bench.py measures real agent processes (env loop + request_for_action + upload), so its
uploads/s is the agents' offered rate.  Here sender processes replay pre-encoded RRLC episode
frames (distinct agent id / seq per frame, CartPole-sized: 4-float obs, 20 rows) through a
native PUSH socket as fast as the server takes them, and the server's ``service.received``
is sampled: what the ZMQ endpoint + learner service (decode, dedupe, hand-off to the learner)
sustain per second.  The learner is the CPU trajectory REINFORCE (``device="cpu"``) with a
large ``traj_per_epoch`` so training does not dominate; ``--engine vec`` on a GPU box feeds the
on-device learner instead.

    python benchmarks/ingest_ceiling.py --senders 4 --seconds 5
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _sender(idx, endpoint, frames_n, rows, ready, go, seconds, out):
    import numpy as np

    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.types import TrajectoryColumns

    rng = np.random.default_rng(idx)
    frames = []
    for s in range(frames_n):
        obs = rng.standard_normal((rows, 4)).astype(np.float32)
        act = rng.integers(0, 2, (rows, 1)).astype(np.int32)
        done = np.zeros(rows, np.uint8)
        done[-1] = 1
        c = TrajectoryColumns(obs, act, np.ones(rows, np.float32), done, np.ones((rows, 2), np.float32),
                              np.full(rows, -0.69, np.float32), f"ingest-{idx}", s)
        frames.append(c.encode())
    push = _native.ZmtpSocket(_native.SockType.PUSH)
    push.connect(endpoint)
    ready.put(idx)
    go.wait()
    stop_at = time.time() + seconds
    sent = 0
    while time.time() < stop_at and sent < frames_n:
        if push.send([frames[sent]], 1000):
            sent += 1
    push.close()
    with open(out, "w") as f:
        json.dump({"sent": sent}, f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--senders", type=int, nargs="*", default=[1, 4, 8])
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--rows", type=int, default=20)
    ap.add_argument("--frames-per-sender", type=int, default=200000,
                    help="pre-encoded episodes per sender; a sender that runs out stops early (reported)")
    ap.add_argument("--engine", default=None, help="None (CPU trajectory learner) or vec (GPU engine)")
    a = ap.parse_args()
    from relayrl_prototype_amd.api.server import TrainingServer
    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
    from relayrl_prototype_amd.utils.addresses import free_port

    for ns in a.senders:
        d = tempfile.mkdtemp(prefix="rrl_ingest_")
        cfg = json.loads(DEFAULT_CONFIG_CONTENT)
        for k in ("training_server", "trajectory_server", "agent_listener"):
            cfg["server"][k]["port"] = str(free_port())
        cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = 1 << 30  # ingest only
        cfgp = os.path.join(d, "relayrl_config.json")
        json.dump(cfg, open(cfgp, "w"))
        kw = {"device": "cpu"} if a.engine is None else {"engine": a.engine}
        srv = TrainingServer("REINFORCE", 4, 2, 1 << 22, env_dir=os.path.join(d, "env"), config_path=cfgp,
                             server_type="zmq", **kw)
        ts = dict(srv.cfg.get_traj_server())
        endpoint = f"tcp://127.0.0.1:{ts['port']}"
        frames_n = int(a.frames_per_sender)
        ctx = mp.get_context("spawn")
        ready, go = ctx.Queue(), ctx.Event()
        outs = [os.path.join(d, f"s{i}.json") for i in range(ns)]
        ps = [ctx.Process(target=_sender, args=(i, endpoint, frames_n, a.rows, ready, go, a.seconds, outs[i]))
              for i in range(ns)]
        for p in ps:
            p.start()
        for _ in range(ns):
            ready.get(timeout=300)
        r0, t0 = srv.service.received, time.perf_counter()
        go.set()
        while time.perf_counter() - t0 < a.seconds:
            time.sleep(0.05)
        r1, t1 = srv.service.received, time.perf_counter()
        for p in ps:
            p.join(60)
        sent = sum(json.load(open(o))["sent"] for o in outs if os.path.exists(o))
        t_drain = time.perf_counter()
        while srv.service.received < r0 + sent and time.perf_counter() - t_drain < 60:
            time.sleep(0.01)
        print(json.dumps({"bench": "ingest_ceiling", "senders": ns, "rows_per_upload": a.rows,
                          "learner": a.engine or "cpu-trajectory", "uploads_per_s_during": round((r1 - r0) / (t1 - t0)),
                          "sent": sent, "senders_exhausted": sent >= ns * frames_n, "received_total": srv.service.received - r0,
                          "drain_s": round(time.perf_counter() - t_drain, 3)}), flush=True)
        srv.close(save=False)


if __name__ == "__main__":
    main()
