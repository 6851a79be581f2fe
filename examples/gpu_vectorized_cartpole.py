#!/usr/bin/env python3
"""Config 2 (BASELINE.json): REINFORCE-with-baseline on CartPole-v1 entirely on one MI355X
-- fused rollout kernel over thousands of envs, HIP value/policy gradient kernels, hipGraph
value loop -- trained until the mean episode return reaches 475 (CartPole-v1 spec).

    python examples/gpu_vectorized_cartpole.py --num-envs 4096
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--num-envs", type=int, default=4096)
    ap.add_argument("--rollout-len", type=int, default=128)
    ap.add_argument("--threshold", type=float, default=475.0)
    ap.add_argument("--max-epochs", type=int, default=200)
    a = ap.parse_args()
    import torch

    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    cfg = VecTrainerConfig(num_envs=a.num_envs, rollout_len=a.rollout_len, pi_lr=1e-2, vf_lr=3e-3,
                           train_vf_iters=20, gamma=0.99, lam=0.95, seed=7)
    tr = VecTrainer(cfg)
    t0 = time.perf_counter()
    for ep in range(a.max_epochs):
        tr.train_epoch()
        m = tr.metrics()
        print(f"epoch {ep + 1}: AverageEpRet {m['AverageEpRet']:.1f}  EnvSteps {m['EnvSteps']}", flush=True)
        if m["AverageEpRet"] >= a.threshold:
            torch.cuda.synchronize()
            print(f"threshold reached in {time.perf_counter() - t0:.3f} s")
            break


if __name__ == "__main__":
    main()
