#!/usr/bin/env python3
"""A2C on PongSynth-v0 pixels (BASELINE.json config 4) -- env steps/s of the full update
(rollout on device + CNN backward + Adam), whole job.  Same launch contract as bench.py:

    python benchmarks/pong_a2c_bench.py --gpus 1 --steps 20 --warmup 3
    torchrun --nproc-per-node 8 benchmarks/pong_a2c_bench.py --gpus 8 ...
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--num-envs", type=int, default=512)
    ap.add_argument("--rollout-len", type=int, default=5)
    ap.add_argument("--phase-timing", action="store_true")
    a = ap.parse_args()
    from relayrl_prototype_amd.parallel.comm import Comm, init_distributed
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    comm = init_distributed() if int(os.environ.get("WORLD_SIZE", "1")) > 1 else Comm()
    from relayrl_prototype_amd.parallel.comm import local_device_index

    dev = torch.device("cuda", local_device_index())
    torch.cuda.set_device(dev)
    cfg = PixelA2CConfig(num_envs=a.num_envs, rollout_len=a.rollout_len, phase_timing=a.phase_timing)
    tr = PixelA2CTrainer(cfg, comm, device=dev)
    for _ in range(a.warmup):
        tr.train_epoch()
    comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_epoch()
    torch.cuda.synchronize()
    comm.barrier()
    el = torch.tensor([time.perf_counter() - t0], device=dev)
    comm.all_reduce_max_(el)
    el = el.item()
    steps = a.steps * a.num_envs * a.rollout_len * comm.world
    m = tr.metrics()
    # data parallel: every rank must hold the same parameters after the all-reduced updates
    sync = None
    if comm.world > 1:
        p = (tr.model.params if tr.on_gpu else tr.params).detach()
        hi, lo = p.clone(), p.clone()
        comm.all_reduce_max_(hi)
        comm.all_reduce_min_(lo)
        sync = bool(torch.equal(hi, lo))
    if comm.rank == 0:
        out = {"metric": "env_steps_per_sec (A2C PongSynth-v0 pixels, Nature-CNN)", "value": steps / el,
               "unit": "env_steps/s", "n_gpus": comm.world, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": el / a.steps * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "bf16 (fp32 accumulate, fp32 master weights)", "data": "synthetic env, random-init weights",
               "config": {"model": "NatureCNN-A2C", "global_batch": a.num_envs * a.rollout_len * comm.world,
                          "seq_len": a.rollout_len, "parallelism": f"dp{comm.world}"},
               "train": {k: m[k] for k in ("AverageEpRet", "Episodes", "LossPi", "LossV", "Entropy")},
               "frame_ring": getattr(tr, "ring", None) is not None}
        if sync is not None:
            out["params_in_sync"] = sync
        if a.phase_timing:
            out["phases_ms"] = tr.timer.columns()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
