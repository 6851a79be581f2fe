#!/usr/bin/env python3
"""Per-env-step cost of the C++ host rollout driver (csrc/runtime/host_rollout.cpp) across
env counts, env threads and wait modes: rollouts only, no learner.  One JSON line each."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="CartPole-v1")
    ap.add_argument("--num-envs", type=int, nargs="*", default=[1024, 8192, 32768])
    ap.add_argument("--threads", type=int, nargs="*", default=[4, 16])
    ap.add_argument("--wait-modes", type=int, nargs="*", default=[0, 1])
    ap.add_argument("--halves", type=int, nargs="*", default=[2])
    ap.add_argument("--T", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for N in a.num_envs:
        for th in a.threads:
            for hv in a.halves:
                for wm in a.wait_modes:
                    cfg = HostTrainerConfig(env=a.env, num_envs=N, rollout_len=a.T, num_threads=th, train_vf_iters=0,
                                            pipeline=hv == 2)
                    tr = HostVecTrainer(cfg, device=dev)
                    tr.driver.set_wait_mode(wm)
                    tr.rollout()
                    torch.cuda.synchronize()
                    tr.driver.take_stats()
                    t0 = time.perf_counter()
                    for _ in range(a.reps):
                        tr.rollout()
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    st = tr.driver.take_stats()
                    n = max(st["steps"], 1)
                    print(json.dumps({"env": a.env, "num_envs": N, "threads": th, "halves": hv, "wait_mode": wm,
                                      "env_steps_per_s": round(N * a.T * a.reps / dt, 1),
                                      "us_per_step": round(dt / (a.T * a.reps) * 1e6, 1),
                                      **{k: round(st[k] / n, 1) for k in ("env_wait_us", "gpu_wait_us", "launch_us")}}),
                          flush=True)
                    tr.close()
                    del tr


if __name__ == "__main__":
    main()
