#!/usr/bin/env python3
"""Sweep the time-to-threshold configuration (CartPole-v1, mean return >= 475) of the
device trainer; one JSON line per (config, seed).  Used to pick bench.py --ttt defaults."""
import itertools
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def ttt(cfg, max_s=20.0, threshold=475.0):
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer

    tr = VecTrainer(cfg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while True:
        tr.train_epoch()
        m = tr.metrics()
        el = time.perf_counter() - t0
        if m["AverageEpRet"] == m["AverageEpRet"] and m["AverageEpRet"] >= threshold:
            return el, tr.epoch, m["EnvSteps"]
        if el > max_s:
            return None, tr.epoch, m["EnvSteps"]


def main():
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainerConfig

    grid = itertools.product([1024, 2048, 4096, 8192], [64, 128], [5, 10, 20], [1e-2, 3e-2])
    for n, t, vfi, lr in grid:
        for seed in (7, 8):
            cfg = VecTrainerConfig(num_envs=n, rollout_len=t, with_baseline=True, pi_lr=lr, vf_lr=3e-3,
                                   train_vf_iters=vfi, gamma=0.99, lam=0.95, seed=seed)
            s, ep, steps = ttt(cfg)
            print(json.dumps({"num_envs": n, "rollout_len": t, "vf_iters": vfi, "pi_lr": lr, "seed": seed,
                              "ttt_s": s, "epochs": ep, "env_steps": steps}), flush=True)


if __name__ == "__main__":
    main()
