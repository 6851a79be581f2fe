#!/usr/bin/env python3
"""Reference-equivalent CPU pipeline, measured on THIS machine (BASELINE.md has no published
numbers, so this is the comparison point for bench.py).

It re-creates the per-step work of the reference's CartPole REINFORCE loop
(SURVEY §3.3 / cartpole_zmq.ipynb):
  * agent: batch-1 TorchScript ``step(obs, mask)`` through the interpreter
    (agent_wrapper.rs, o3_agent.rs request_for_action), safetensors encodes of
    obs / act / mask / aux per action (action.rs:40-90);
  * upload: the episode as one pickle of per-action dicts (trajectory.rs:50-55), decoded
    and re-parsed per action on the learner (python_algorithm_request.rs ->
    REINFORCE.receive_trajectory);
  * learner: PyTorch-CPU REINFORCE with value baseline, traj_per_epoch=8, one policy step
    and 80 value iterations (REINFORCE.py:97-147), then a TorchScript re-export
    (REINFORCE.py:64-68) every epoch.
Transport is in-process (no sockets), which only flatters the reference.  Pickle is
used on data this script generates itself.

    python benchmarks/reference_equivalent_cpu.py --seconds 60
"""
import argparse
import io
import json
import os
import pickle
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--threshold", type=float, default=475.0)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--window", type=int, default=100,
                    help="solved = mean return of the newest `window` finished episodes >= threshold (gymnasium "
                         "CartPole-v1: 100), checked after every epoch like bench.py")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    from relayrl_prototype_amd import _native
    from relayrl_prototype_amd.models.policies import build_policy_module
    from relayrl_prototype_amd.ops.mlp import MLPSpec

    D, A, H = 4, 2, 128
    gamma, lam, traj_per_epoch, vf_iters = 0.98, 0.97, 8, 80
    torch.manual_seed(1)
    pi = MLPSpec(D, H, A).init()
    vf = MLPSpec(D, H, 1).init()
    model = build_policy_module(D, A, H, pi, vf, True)
    pi_net, v_net = model.policy.pi_network, model.baseline.v_network
    opt_pi = torch.optim.Adam(pi_net.parameters(), lr=3e-4)
    opt_vf = torch.optim.Adam(v_net.parameters(), lr=1e-3)

    def export():
        buf = io.BytesIO()
        torch.jit.save(torch.jit.script(model), buf)
        buf.seek(0)
        return torch.jit.load(buf)

    scripted = export()
    env = _native.VecEnv("CartPole-v1", 1, 0, 1)
    obs = np.zeros((1, D), np.float32)
    rew = np.zeros(1, np.float32)
    done = np.zeros(1, np.float32)
    act = np.zeros(1, np.int32)
    env.reset_ptr(obs.ctypes.data)
    mask_t = torch.ones(1, A)
    episodes, steps, ep_actions, ep_rets, best_avg = [], 0, [], [], 0.0
    ttt = None
    t0 = time.perf_counter()
    epoch_rets = []
    while time.perf_counter() - t0 < a.seconds:
        o = torch.from_numpy(obs.copy())
        with torch.no_grad():
            at, data = scripted.step(o, mask_t)
        act[0] = int(at.reshape(-1)[0])
        rec = {"obs": _native.st_encode("Float", [D], obs.tobytes()),
               "act": _native.st_encode("Int", [1], act.tobytes()),
               "mask": _native.st_encode("Float", [A], mask_t.numpy().tobytes()),
               "data": {k: _native.st_encode("Float", [1], v.numpy().astype(np.float32).tobytes())
                        for k, v in data.items()}}
        env.step_ptr(act.ctypes.data, obs.ctypes.data, rew.ctypes.data, done.ctypes.data)
        rec["rew"] = float(rew[0])
        rec["done"] = bool(done[0] > 0)
        ep_actions.append(rec)
        steps += 1
        if done[0] > 0:
            episodes.append(pickle.dumps(ep_actions))
            ep_actions = []
            if len(episodes) == traj_per_epoch:
                O, Ac, R, DONE = [], [], [], []
                for e in episodes:  # learner: unpickle + per-action decode
                    for r in pickle.loads(e):
                        O.append(np.frombuffer(_native.st_decode(r["obs"])[2], np.float32))
                        Ac.append(np.frombuffer(_native.st_decode(r["act"])[2], np.int32)[0])
                        R.append(r["rew"])
                        DONE.append(r["done"])
                episodes = []
                O = torch.from_numpy(np.stack(O))
                Ac = torch.tensor(Ac, dtype=torch.long)
                R = np.asarray(R, np.float32)
                DONE = np.asarray(DONE)
                with torch.no_grad():
                    V = v_net(O)[:, 0].numpy()
                adv = np.zeros_like(R)
                ret = np.zeros_like(R)
                la, rr = 0.0, 0.0
                ep_ret = 0.0
                for t in range(len(R) - 1, -1, -1):
                    nv = 0.0 if DONE[t] else V[t + 1]
                    if DONE[t]:
                        la, rr = 0.0, 0.0
                    delta = R[t] + gamma * nv - V[t]
                    la = delta + gamma * lam * la
                    rr = R[t] + gamma * rr
                    adv[t], ret[t] = la, rr
                s = 0.0
                for t in range(len(R)):
                    s += R[t]
                    if DONE[t]:
                        epoch_rets.append(s)
                        s = 0.0
                adv_t = torch.from_numpy((adv - adv.mean()) / (adv.std() + 1e-8))
                logp = torch.log_softmax(pi_net(O), -1).gather(1, Ac[:, None])[:, 0]
                opt_pi.zero_grad()
                (-(logp * adv_t).mean()).backward()
                opt_pi.step()
                ret_t = torch.from_numpy(ret)
                for _ in range(vf_iters):
                    opt_vf.zero_grad()
                    ((v_net(O)[:, 0] - ret_t) ** 2).mean().backward()
                    opt_vf.step()
                scripted = export()
                if len(epoch_rets) >= a.window:
                    avg = float(np.mean(epoch_rets[-a.window:]))
                    best_avg = max(best_avg, avg)
                    if ttt is None and avg >= a.threshold:
                        ttt = time.perf_counter() - t0
                        break
            env.reset_ptr(obs.ctypes.data)
    el = time.perf_counter() - t0
    print(json.dumps({"metric": "env_steps_per_sec (reference-equivalent CPU pipeline)", "value": steps / el,
                      "unit": "env_steps/s", "seconds": el, "env_steps": steps, "episodes": len(epoch_rets),
                      "best_window_return": best_avg, "window": a.window, "time_to_threshold_s": ttt,
                      "threshold": a.threshold, "torch_threads": a.threads}))


if __name__ == "__main__":
    main()
