#!/usr/bin/env python3
"""The reference notebooks' flow as a script (examples/REINFORCE_*/**/{zmq,grpc}/*.ipynb):
a TrainingServer and a RelayRLAgent in one process, an env loop calling
request_for_action / flag_last_action, the learner updating every traj_per_epoch
episodes and pushing new weights to the agent.

    python examples/agent_server_loop.py --env CartPole-v1 --server-type zmq --episodes 200
    python examples/agent_server_loop.py --env LunarLanderSynth-v0 --server-type grpc --with-baseline

Envs come from the C++ VecEnv (gymnasium is not installed): CartPole-v1, MountainCar-v0,
Acrobot-v1, Pendulum-v1, LunarLanderSynth-v0, HalfCheetahSynth-v0.
"""
import argparse
import json
import os
import socket
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="CartPole-v1")
    ap.add_argument("--server-type", default="zmq", choices=["zmq", "grpc", "local"])
    ap.add_argument("--episodes", type=int, default=100)
    ap.add_argument("--with-baseline", action="store_true")
    ap.add_argument("--algorithm", default="REINFORCE", choices=["REINFORCE", "PPO", "A2C"])
    ap.add_argument("--traj-per-epoch", type=int, default=8)
    ap.add_argument("--dir", default=None, help="env_dir for logs / models (default: a temp dir)")
    a = ap.parse_args()

    from relayrl_prototype_amd import RelayRLAgent, TrainingServer, _native
    from relayrl_prototype_amd.config import DEFAULT_CONFIG_CONTENT

    env_dir = a.dir or tempfile.mkdtemp(prefix="relayrl_")
    cfg = json.loads(DEFAULT_CONFIG_CONTENT)
    for k in ("training_server", "trajectory_server", "agent_listener"):
        cfg["server"][k]["port"] = str(free_port())
    cfg_path = os.path.join(env_dir, "relayrl_config.json")
    json.dump(cfg, open(cfg_path, "w"), indent=2)

    env = _native.VecEnv(a.env, 1, 0, 1)
    D, A, cont = env.obs_dim, env.act_dim, env.continuous
    hp = {"traj_per_epoch": str(a.traj_per_epoch), "with_vf_baseline": str(a.with_baseline).lower(),
          "discrete": str(not cont).lower()}
    server = TrainingServer(a.algorithm, D, A, 1_000_000, env_dir=env_dir, config_path=cfg_path,
                            server_type=a.server_type, hyperparams=hp)
    agent = RelayRLAgent(config_path=cfg_path, server_type=a.server_type)
    obs = np.zeros((1, D), np.float32)
    rew = np.zeros(1, np.float32)
    done = np.zeros(1, np.float32)
    act = np.zeros((1, A), np.float32) if cont else np.zeros(1, np.int32)
    env.reset_ptr(obs.ctypes.data)
    returns = []
    for ep in range(a.episodes):
        r, ret = 0.0, 0.0
        while True:
            action = agent.request_for_action(obs[0], None, r)
            act[...] = np.asarray(action.get_act()).reshape(act.shape[1:] if cont else ())
            env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
            r = float(rew[0])
            ret += r
            if done[0] > 0:
                agent.flag_last_action(r)
                break
        returns.append(ret)
        if (ep + 1) % 10 == 0:
            print(f"episode {ep + 1}: mean return (last 10) {np.mean(returns[-10:]):.1f}  "
                  f"model version {agent.model_version}", flush=True)
    server.wait_idle(60)
    print(json.dumps({"episodes": len(returns), "updates": server.service.updates, "env_dir": env_dir}))
    agent.close()
    server.close()


if __name__ == "__main__":
    main()
