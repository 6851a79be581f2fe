#!/usr/bin/env python3
"""Many concurrent agent PROCESSES fanning in to one TrainingServer -- the reference's actual
distribution mode (N agents -> one PULL, trajectory.rs:69-90 with a new connection per
upload; training_zmq.rs:948-1058) -- and the reference's paced protocol
(network_benchmarks.rs:20,283-284,368-369: NEXT_ACTION_WAIT_MILLIS between actions,
TRAJECTORY_SIZES actions per upload).

One row per (transport, agents, wait_ms):

  transport  zmq          native RRLC frames over one persistent PUSH per agent
             zmq-ref      the reference agent's wire: serde_pickle(Vec<RelayRLAction>) frames,
                          a NEW TCP connection + ZMTP handshake per upload (trajectory.rs:69-90)
             grpc         unary SendActions with RRLC frames
  learner    engine       (GPU) TrainingServer(engine="vec"): the uploads are folded into the
                          on-device learner's epochs (runtime/engine.py agent rows) while it
                          trains in the background
             trajectory   (CPU) the trajectory learner (REINFORCE, algorithms/trajectory_algo.py)

Reported: uploads/s the learner service processed while the agents ran, agent env steps/s,
ingestion lag (agent send -> learner service processed, p50 / p99, native wire: matched on
(agent id, episode seq)), the backlog at the stop and the time to drain it, drops (sent -
received after the drain, plus the learner's own rejections), and the server's thread count
before / during / after (the ZMTP server serves every connection from one I/O thread).

    python benchmarks/fanin_bench.py --agents 16 64 --transports zmq zmq-ref grpc --seconds 10
    python benchmarks/fanin_bench.py --agents 16 --paced 25 50 100 --traj-size 10
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

NEXT_ACTION_WAIT_MILLIS = [1000, 750, 500, 333, 250, 100, 50, 25]  # network_benchmarks.rs:20
TRAJECTORY_SIZES = [10, 50, 100, 250, 500, 1000]                  # network_benchmarks.rs:19


def _agent_main(idx, cfg_path, transport, wait_ms, traj_size, start_at, stop_at, out_path, train_port):
    """One agent process: CartPole (C++ env) with ``traj_size`` 0, else the reference bench's
    fixed-size episodes of constant observations; ``wait_ms`` between actions."""
    import numpy as np

    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.api.agent import RelayRLAgent

    os.environ["RRL_QUIET_CONFIG"] = "1"
    st = {"zmq": "zmq", "zmq-ref": "zmq", "grpc": "grpc"}[transport]
    wire = "reference" if transport == "zmq-ref" else "columns"
    kw = {"connection_per_upload": True, "training_port": str(train_port)} if transport == "zmq-ref" else {}
    for attempt in range(5):
        try:
            agent = RelayRLAgent(config_path=cfg_path, server_type=st, wire_format=wire, agent_id=f"fanin-{idx}",
                                 seed=idx, **kw)
            break
        except RuntimeError as e:
            # a reference agent binds its own PULL port; the parent's free_port() can be taken
            # again (by another agent's outgoing connection) before the child binds it
            if transport != "zmq-ref" or "already in use" not in str(e) or attempt == 4:
                raise
            from relayrl_prototype_amd.utils.addresses import free_port

            kw["training_port"] = str(free_port())
    env = _native.VecEnv("CartPole-v1", 1, 1000 + idx, 1)
    o = np.zeros((1, 4), np.float32)
    r = np.zeros(1, np.float32)
    d = np.zeros(1, np.float32)
    a = np.zeros(1, np.int32)
    env.reset_ptr(o.ctypes.data)
    mask = np.ones(2, np.float32)
    sends, steps, rew, n_in_ep = [], 0, 0.0, 0
    while time.time() < start_at:
        time.sleep(0.001)
    while time.time() < stop_at:
        act = agent.request_for_action(o[0], mask, rew)
        steps += 1
        n_in_ep += 1
        if traj_size:
            rew = 1.0
            done = n_in_ep >= traj_size
        else:
            a[0] = int(np.asarray(act.get_act()).reshape(-1)[0])
            env.step_ptr(a.ctypes.data, o.ctypes.data, r.ctypes.data, d.ctypes.data)
            rew = float(r[0])
            done = d[0] > 0
        if done:
            seq = agent.episodes_sent
            t = time.time()
            agent.flag_last_action(rew)
            sends.append((seq, t, time.time() - t, n_in_ep))
            rew, n_in_ep = 0.0, 0
        if wait_ms:
            time.sleep(wait_ms / 1000.0)
    agent.close()
    with open(out_path, "w") as f:
        json.dump({"idx": idx, "steps": steps, "sends": sends}, f)


def _config(tmp):
    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
    from relayrl_prototype_amd.utils.addresses import free_port

    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = 64
    cfg["algorithms"]["REINFORCE"]["with_vf_baseline"] = True
    cfg["max_traj_length"] = 4096
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    p = os.path.join(tmp, "relayrl_config.json")
    with open(p, "w") as f:
        json.dump(cfg, f)
    return p


def run(transport, n_agents, seconds, wait_ms, traj_size, learner) -> dict:
    from relayrl_prototype_amd.api.server import TrainingServer
    from relayrl_prototype_amd.utils.addresses import free_port

    os.environ["RRL_QUIET_CONFIG"] = "1"
    tmp = tempfile.mkdtemp()
    cfgp = _config(tmp)
    st = "grpc" if transport == "grpc" else "zmq"
    threads = lambda: len(os.listdir("/proc/self/task"))  # noqa: E731
    kw = {}
    if learner == "engine":
        kw = dict(engine="vec", hyperparams={"num_envs": 4096, "rollout_len": 32, "train_vf_iters": 20,
                                             "agent_rows_cap": 1 << 18})
    else:
        kw = dict(device="cpu")
    srv = TrainingServer("REINFORCE", 4, 2, 1 << 20, env_dir=tmp, config_path=cfgp, server_type=st, **kw)
    # ingestion timestamps (native wire: agent id + episode seq)
    done_at = {}
    proc = srv.service.process

    def timed(traj):
        out = proc(traj)
        aid = getattr(traj, "agent_id", "")
        if aid:
            done_at[(aid, int(getattr(traj, "seq", -1)))] = time.time()
        return out

    srv.service.process = timed
    th0 = threads()
    if learner == "engine":
        srv.train(max_seconds=seconds + 60, log_every=0, publish_every=1, background=True)
    ctx = mp.get_context("spawn")
    start_at = time.time() + 8.0 + 0.15 * n_agents  # every agent process imported + handshaken
    stop_at = start_at + seconds
    outs = [os.path.join(tmp, f"agent{i}.json") for i in range(n_agents)]
    ps = [ctx.Process(target=_agent_main, args=(i, cfgp, transport, wait_ms, traj_size, start_at, stop_at, outs[i],
                                                free_port() if transport == "zmq-ref" else 0))
          for i in range(n_agents)]
    for p in ps:
        p.start()
    th_peak = th0
    while time.time() < stop_at:
        th_peak = max(th_peak, threads())
        time.sleep(0.05)
    received_in_window = srv.service.received  # processed while the agents were running
    for p in ps:
        p.join(timeout=120)
    t_agents_done = time.time()
    rows = []
    for o in outs:
        try:
            rows.append(json.load(open(o)))
        except (OSError, ValueError):
            pass
    sent = sum(len(r["sends"]) for r in rows)
    # drain: uploads still in the socket inbox / decode / service queue at the stop
    backlog = sent - srv.service.received
    last, t_change = -1, time.time()
    while time.time() - t_agents_done < 120:
        r = srv.service.received
        if r >= sent:
            break
        if r != last:
            last, t_change = r, time.time()
        elif time.time() - t_change > 10:
            break  # no progress: the rest is lost
        time.sleep(0.01)
    drained = srv.wait_idle(60) and srv.service.received >= sent
    drain_s = time.time() - t_agents_done
    received = srv.service.received
    steps = sum(r["steps"] for r in rows)
    lags, send_ms = [], []
    for r in rows:
        for seq, t, dt, _ in r["sends"]:
            send_ms.append(dt * 1e3)
            k = (f"fanin-{r['idx']}", int(seq))
            if k in done_at:
                lags.append((done_at[k] - t) * 1e3)
    lags.sort()
    send_ms.sort()
    pct = lambda v, q: round(v[min(len(v) - 1, int(q * len(v)))], 3) if v else None  # noqa: E731
    algo = srv.algorithm
    rejected = int(getattr(algo, "ignored_trajectories", 0))
    res = {"transport": transport, "agents": n_agents, "learner": learner, "wait_ms": wait_ms,
           "traj_size": traj_size or "cartpole", "seconds": seconds, "agent_processes_ok": len(rows),
           "uploads_sent": sent, "uploads_received": received, "drops": sent - received, "learner_rejected": rejected,
           "uploads_per_s": round(received_in_window / seconds, 1), "backlog_at_stop": backlog,
           "agent_env_steps_per_s": round(steps / seconds, 1),
           "send_call_ms_p50": pct(send_ms, 0.5), "send_call_ms_p99": pct(send_ms, 0.99),
           "ingest_lag_ms_p50": pct(lags, 0.5), "ingest_lag_ms_p99": pct(lags, 0.99), "lag_samples": len(lags),
           "drain_s": round(drain_s, 3), "drained": drained, "server_threads": [th0, th_peak, threads()]}
    if learner == "engine":
        srv.engine.stop()
        r = srv.engine.join(120)
        res.update(engine_epochs=None if r is None else r.epochs, agent_rows_folded=int(algo.agent_rows_total),
                   agent_episodes_folded=int(algo.agent_episodes))
    srv.close(save=False)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--agents", type=int, nargs="+", default=[16, 64])
    ap.add_argument("--transports", nargs="+", default=["zmq", "zmq-ref", "grpc"])
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--paced", type=int, nargs="*", default=[0],
                    help="ms between an agent's actions (the reference's NEXT_ACTION_WAIT_MILLIS); 0 = unpaced")
    ap.add_argument("--traj-size", type=int, default=0,
                    help="actions per upload (the reference's TRAJECTORY_SIZES); 0 = CartPole episodes")
    ap.add_argument("--learner", choices=("auto", "engine", "trajectory"), default="auto")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    learner = a.learner
    if learner == "auto":
        import torch

        learner = "engine" if torch.cuda.is_available() else "trajectory"
    for t in a.transports:
        for n in a.agents:
            for w in a.paced:
                line = json.dumps(run(t, n, a.seconds, w, a.traj_size, learner))
                print(line, flush=True)
                if a.out:
                    with open(a.out, "a") as f:
                        f.write(line + "\n")


if __name__ == "__main__":
    main()
