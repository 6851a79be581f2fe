#!/usr/bin/env python3
"""Rollout time of the C++ host driver while learner kernels run concurrently, by stream
setup (which streams, CU masks, priorities).  Finds what makes the overlapped host-env
trainer's sampling launches wait for the learner."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch


def main():
    from relayrl_prototype_amd.ops import GradHead, grad_slabs, hip, mlp_grad, MLPSpec
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    h = hip()
    n = h.device_cus()
    B = 524288
    spec = MLPSpec(4, 128, 1)
    vp = spec.init(torch.Generator().manual_seed(0)).to(dev)
    obs = torch.randn(B, 4, device=dev)
    ret = torch.randn(B, device=dev)

    def learner_burst(iters, stream):
        with torch.cuda.stream(stream):
            ns = grad_slabs(B, dev)
            slab = torch.empty(ns, spec.P, device=dev)
            ls = torch.empty(ns, 8, device=dev)
            for _ in range(iters):
                mlp_grad(GradHead.VALUE_MSE, vp, obs, 1, 128, ret=ret, inv_B=1.0 / B, grad_slab=slab, loss_slab=ls)

    cfg = HostTrainerConfig(env="CartPole-v1", num_envs=8192, rollout_len=64, num_threads=16, train_vf_iters=0)
    tr = HostVecTrainer(cfg, device=dev)
    tr.rollout()
    torch.cuda.synchronize()
    # CU-mask bit i lands on XCC i % 8 (KFD spreads mask bits round-robin over the XCCs), so
    # bits 0..15 = 2 CUs per XCD; a stride-16 pick would put all 16 on one XCD
    actor_cus = list(range(16))
    learner_cus = [c for c in range(n) if c not in set(actor_cus)]
    stride_actor = [i * (n // 16) for i in range(16)]
    stride_learner = [c for c in range(n) if c not in set(stride_actor)]
    setups = {
        "no_learner": (None, torch.cuda.current_stream()),
        "learner_alone": ("alone", None),
        "same_stream": ("same", torch.cuda.current_stream()),
        "side_stream": (torch.cuda.Stream(), torch.cuda.current_stream()),
        "side_stream_hiprio_actor": (torch.cuda.Stream(), torch.cuda.Stream(priority=-1)),
        "masked_both": (torch.cuda.ExternalStream(h.cu_masked_stream(learner_cus)),
                        torch.cuda.ExternalStream(h.cu_masked_stream(actor_cus))),
        "masked_actor_only": (torch.cuda.Stream(), torch.cuda.ExternalStream(h.cu_masked_stream(actor_cus))),
        "masked_both_stride": (torch.cuda.ExternalStream(h.cu_masked_stream(stride_learner)),
                               torch.cuda.ExternalStream(h.cu_masked_stream(stride_actor))),
    }
    for name, (lstream, astream) in setups.items():
        for limit in ([0, len(learner_cus)] if name.startswith("masked_both") else [0]):
            h.set_cu_limit(limit)
            torch.cuda.synchronize()
            tr.driver.take_stats()
            t0 = time.perf_counter()
            if lstream is not None:
                learner_burst(80, torch.cuda.current_stream() if lstream in ("same", "alone") else lstream)
            if astream is not None:
                with torch.cuda.stream(astream):
                    tr.rollout()
            t_roll = time.perf_counter() - t0
            torch.cuda.synchronize()
            t_all = time.perf_counter() - t0
            st = tr.driver.take_stats()
            k = max(st["steps"], 1)
            print(json.dumps({"setup": name, "cu_limit": limit, "rollout_ms": round(t_roll * 1e3, 2),
                              "total_ms": round(t_all * 1e3, 2),
                              "gpu_wait_us_per_step": round(st["gpu_wait_us"] / k, 1),
                              "env_wait_us_per_step": round(st["env_wait_us"] / k, 1)}), flush=True)
    h.set_cu_limit(0)
    tr.close()


if __name__ == "__main__":
    main()
