#!/usr/bin/env python3
"""Time-to-threshold with and without the hipGraph-captured value loop: trainer construction
time, TTT, first-epoch and median epoch time (median over 10 seeds, bench.py's TTT config)."""
import sys, time, json, statistics
sys.path.insert(0, '.')
import torch
from relayrl_prototype_amd.runtime.vec_trainer import SolvedCheck, VecTrainer, VecTrainerConfig
torch.cuda.set_device(0)
def one(seed, graphs):
    torch.cuda.synchronize(); tc = time.perf_counter()
    cfg = VecTrainerConfig(num_envs=1024, rollout_len=64, with_baseline=True, pi_lr=1e-2, vf_lr=1e-2,
                           train_vf_iters=5, gamma=0.99, lam=0.95, seed=seed, use_graphs=graphs)
    tr = VecTrainer(cfg); torch.cuda.synchronize(); t0 = time.perf_counter()
    chk = SolvedCheck(475.0, 100); ep_t = []
    while True:
        te = time.perf_counter(); tr.train_epoch(); r = chk.update(*tr.episode_sums()); ep_t.append(time.perf_counter() - te)
        if chk.solved(r) or time.perf_counter() - t0 > 2: break
    return {"construct_ms": (t0 - tc) * 1e3, "ttt_ms": (time.perf_counter() - t0) * 1e3, "epochs": tr.epoch,
            "first_epoch_ms": ep_t[0] * 1e3, "median_epoch_ms": statistics.median(ep_t) * 1e3}
one(99, True); one(99, False)
for g in (True, False):
    res = [one(s, g) for s in range(1, 11)]
    print(json.dumps({"graphs": g, **{k: round(statistics.median(r[k] for r in res), 3) for k in res[0]}}))
