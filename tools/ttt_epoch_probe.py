#!/usr/bin/env python3
"""Where does a time-to-threshold epoch go?  Times 30 epochs of the bench.py TTT config
(1024 envs x 64 steps, 10 value iterations) three ways: with the per-epoch threshold read,
without any per-epoch read (GPU-queue bound), and the summed per-phase HIP-event times."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig


REF = "--ref" in sys.argv  # the reference hyperparameters (80 value iterations per epoch)
# --shape N T: envs x rollout length (default 1024 x 64)
SHAPE = (int(sys.argv[sys.argv.index("--shape") + 1]), int(sys.argv[sys.argv.index("--shape") + 2])) \
    if "--shape" in sys.argv else (1024, 64)


def cfg(**kw):
    if REF:
        return VecTrainerConfig(num_envs=SHAPE[0], rollout_len=SHAPE[1], with_baseline=True, pi_lr=3e-4, vf_lr=1e-3,
                                train_vf_iters=80, gamma=0.98, lam=0.97, seed=1, **kw)
    return VecTrainerConfig(num_envs=SHAPE[0], rollout_len=SHAPE[1], with_baseline=True, pi_lr=1e-2, vf_lr=3e-3,
                            train_vf_iters=10, gamma=0.99, lam=0.95, seed=1, **kw)


def run(read_each, E=30, **kw):
    tr = VecTrainer(cfg(**kw))
    for _ in range(3):
        tr.train_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(E):
        tr.train_epoch()
        if read_each:
            tr.average_ep_return()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / E * 1e3, tr


out = {}
out["ms_per_epoch_with_read"] = run(True)[0]
out["ms_per_epoch_no_read"] = run(False)[0]
ms, tr = run(False, phase_timing=True)
cols = tr.metrics()
out["phase_cols"] = {k: v for k, v in cols.items() if k.endswith("Ms") or "Time" in k}
print(json.dumps(out))
