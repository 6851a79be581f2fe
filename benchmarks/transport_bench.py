#!/usr/bin/env python3
"""Agent <-> training-server transport benchmarks (reference benches T1:
rf/benches/network_benchmarks.rs -- defined but never runnable there).

Measures, for server_type in local / zmq / grpc:
  * inference latency of request_for_action at batch 1 (CPU policy from flat weights);
  * episode upload latency (flag_last_action) for TRAJECTORY_SIZES = 10..1000 actions;
  * end-to-end single-agent env steps/s on the C++ CartPole with learning disabled.
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np

TRAJECTORY_SIZES = [10, 50, 100, 250, 500, 1000]


def bench(server_type, reps=200, wire="columns"):
    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.api.agent import RelayRLAgent
    from relayrl_prototype_amd.api.server import TrainingServer
    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT
    from relayrl_prototype_amd.utils.addresses import free_port

    tmp = tempfile.mkdtemp()
    os.chdir(tmp)
    os.environ["RRL_QUIET_CONFIG"] = "1"
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    cfg["algorithms"]["REINFORCE"]["traj_per_epoch"] = 10 ** 9  # no training during the bench
    cfg["max_traj_length"] = 4096
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    cfgp = os.path.join(tmp, "relayrl_config.json")
    open(cfgp, "w").write(json.dumps(cfg))
    srv = TrainingServer("REINFORCE", 4, 2, 10 ** 6, env_dir=tmp, config_path=cfgp, server_type=server_type,
                         device="cpu")
    agent = RelayRLAgent(config_path=cfgp, server_type=server_type, wire_format=wire)
    obs = np.zeros(4, np.float32)
    mask = np.ones(2, np.float32)
    out = {"server_type": server_type, "wire_format": wire}
    for _ in range(20):
        agent.request_for_action(obs, mask, 0.0)
    agent.clear_episode()
    t0 = time.perf_counter()
    for _ in range(reps):
        agent.request_for_action(obs, mask, 1.0)
    out["inference_us"] = (time.perf_counter() - t0) / reps * 1e6
    agent.clear_episode()
    lat = {}
    for n in TRAJECTORY_SIZES:
        ts = []
        for _ in range(5):
            for _ in range(n):
                agent.request_for_action(obs, mask, 1.0)
            t0 = time.perf_counter()
            agent.flag_last_action(1.0)
            ts.append(time.perf_counter() - t0)
        lat[n] = sorted(ts)[len(ts) // 2] * 1e6
    out["upload_us_by_traj_size"] = lat
    env = _native.VecEnv("CartPole-v1", 1, 0, 1)
    o = np.zeros((1, 4), np.float32)
    r = np.zeros(1, np.float32)
    d = np.zeros(1, np.float32)
    a = np.zeros(1, np.int32)
    env.reset_ptr(o.ctypes.data)
    steps, t0, rew = 0, time.perf_counter(), 0.0
    while time.perf_counter() - t0 < 2.0:
        act = agent.request_for_action(o[0], mask, rew)
        a[0] = int(np.asarray(act.get_act()).reshape(-1)[0])
        env.step_ptr(a.ctypes.data, o.ctypes.data, r.ctypes.data, d.ctypes.data)
        rew = float(r[0])
        steps += 1
        if d[0] > 0:
            agent.flag_last_action(rew)
            rew = 0.0
    out["single_agent_env_steps_per_s"] = steps / (time.perf_counter() - t0)
    srv.wait_idle(30)
    out["server_received"] = srv.service.received
    agent.close()
    srv.close(save=False)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--types", nargs="*", default=["local", "zmq", "grpc"])
    ap.add_argument("--wire", nargs="*", default=["columns", "actions"],
                    help="columns | actions | reference (the reference agent's own wire)")
    a = ap.parse_args()
    for t in a.types:
        for w in a.wire:
            if t == "local" and w == "actions":
                continue
            print(json.dumps(bench(t, wire=w)), flush=True)


if __name__ == "__main__":
    main()
