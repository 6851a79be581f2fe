#!/usr/bin/env python3
"""BASELINE config #5 at full scale: PPO HalfCheetah (continuous Gaussian policy) with a
>= 10^8-transition rollout buffer resident in one MI355X's HBM.

65,536 envs x 2,048 steps = 134 M transitions per epoch: obs / pre-reset obs buffers of
9.1 GB each, actions 3.2 GB, the scan and learner buffers beside them.  The rollout kernel,
the value forward, the GAE scan and the fused PPO policy / value steps all run on the whole
buffer; the fwd+bwd launches are chunked at ops.mlp.GRAD_CHUNK_ROWS rows (32-bit row x
feature indexing inside the kernels), their slabs summed by one fused reduce + Adam.

After the timed epochs the GAE scan is re-checked in float64 on the CPU for randomly
sampled env columns of the big buffer (the oracle of ops/reference.py), and the JSON line
reports env-steps/s, the buffer sizes and the peak HBM in use.
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
    ap.add_argument("--num-envs", type=int, default=65536)
    ap.add_argument("--rollout-len", type=int, default=2048)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--pi-iters", type=int, default=10)
    ap.add_argument("--vf-iters", type=int, default=10)
    ap.add_argument("--check-cols", type=int, default=64)
    a = ap.parse_args()
    from relayrl_prototype_amd.ops import mlp as mlpops
    from relayrl_prototype_amd.ops import reference as ref
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = VecTrainerConfig(env="HalfCheetahSynth-v0", algo="ppo", num_envs=a.num_envs, rollout_len=a.rollout_len,
                           train_pi_iters=a.pi_iters, train_vf_iters=a.vf_iters, gamma=0.99, lam=0.95,
                           with_baseline=True, use_graphs=False)
    t_alloc = time.perf_counter()
    tr = VecTrainer(cfg)
    torch.cuda.synchronize()
    t_alloc = time.perf_counter() - t_alloc
    for _ in range(a.warmup):
        tr.train_epoch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        tr.train_epoch()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    m = tr.metrics()
    # scan oracle on sampled columns of the newest rollout (float64, CPU)
    T, N = a.rollout_len, a.num_envs
    g = torch.Generator().manual_seed(0)
    cols = torch.randperm(N, generator=g)[:a.check_cols].to(dev)
    rl = tr.rl
    rew = tr.rew[:, cols].double().cpu()
    done = tr.done[:, cols].double().cpu()
    val = rl.val.view(T + 1, N)[:, cols].double().cpu()
    tval = rl.tval[:, cols].double().cpu()
    a_ref, r_ref, _ = ref.gae_scan_tm_ref(rew, done, val.reshape(-1), 0.99, 0.95, tval)
    a_dev, r_dev = rl.adv[:, cols].double().cpu(), rl.ret[:, cols].double().cpu()
    err_adv = float((a_dev - a_ref).abs().max() / a_ref.abs().max().clamp(min=1e-12))
    err_ret = float((r_dev - r_ref).abs().max() / r_ref.abs().max().clamp(min=1e-12))
    transitions = T * N
    buf_gb = sum(t.numel() * t.element_size() for t in (tr.obs, tr.act, tr.logp, tr.rew, tr.done, tr.tobs, rl.val,
                                                         rl.tval, rl.adv, rl.ret)) / 2 ** 30
    print(json.dumps({
        "bench": "big_buffer_ppo_halfcheetah", "baseline_config": 5, "transitions_per_epoch": transitions,
        "num_envs": N, "rollout_len": T, "env_steps_per_s": round(transitions * a.steps / dt, 1),
        "s_per_epoch": round(dt / a.steps, 3), "alloc_s": round(t_alloc, 2), "rollout_buffers_gb": round(buf_gb, 2),
        "hbm_peak_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
        "grad_launches_per_step": len(mlpops.grad_chunks(transitions)), "grad_chunk_rows": mlpops.GRAD_CHUNK_ROWS,
        "scan_oracle_cols": a.check_cols, "scan_rel_err_adv": err_adv, "scan_rel_err_ret": err_ret,
        "avg_ep_ret": m.get("AverageEpRet"), "loss_pi": m.get("LossPi"), "loss_v": m.get("LossV"),
        "dtype": "fp32 (bf16x6 split MFMA learner)", "data": "synthetic HalfCheetahSynth-v0 (docs/ENVS.md)"}),
        flush=True)
    assert err_adv < 1e-4 and err_ret < 1e-4, (err_adv, err_ret)


if __name__ == "__main__":
    main()
