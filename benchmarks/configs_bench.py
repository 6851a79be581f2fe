#!/usr/bin/env python3
"""Throughput of every BASELINE.json configuration preset (runtime/launcher.py PRESETS)
on the current node: W untimed epochs, then K timed epochs bracketed by barrier +
synchronize; one JSON line per preset (whole-job env steps/s).

    python benchmarks/configs_bench.py --presets lunarlander-reinforce-baseline halfcheetah-ppo --steps 5
    torchrun --nproc-per-node 8 benchmarks/configs_bench.py --presets pong-a2c
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
    ap.add_argument("--presets", nargs="*", default=["cartpole-reinforce-baseline", "lunarlander-reinforce-baseline",
                                                     "pong-a2c", "halfcheetah-ppo"])
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--set", nargs="*", default=[])
    a = ap.parse_args()
    from relayrl_prototype_amd.parallel.comm import Comm, dist_env, init_distributed
    from relayrl_prototype_amd.runtime.launcher import PRESETS, _epoch, _make_trainer

    from relayrl_prototype_amd.parallel.comm import local_device_index

    _, _, world = dist_env()
    comm = init_distributed() if world > 1 else Comm()
    dev = torch.device("cuda", local_device_index()) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    ov = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        ov[k] = json.loads(v)
    for name in a.presets:
        p = PRESETS[name]
        if p.kind == "agent_server":
            continue
        tr = _make_trainer(p, comm, dev, ov)
        for _ in range(a.warmup):
            _epoch(tr)
        m0 = tr.metrics()
        comm.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            _epoch(tr)
        if hasattr(tr, "finish"):
            tr.finish()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
        el = torch.tensor([time.perf_counter() - t0], device=dev)
        comm.all_reduce_max_(el)
        m1 = tr.metrics()
        if comm.rank == 0:
            steps = m1.get("EnvSteps", 0) - m0.get("EnvSteps", 0)
            print(json.dumps({"preset": name, "baseline_config": p.baseline_config, "n_gpus": comm.world,
                              "env_steps_per_sec": steps / el.item(), "ms_per_epoch": el.item() / a.steps * 1e3,
                              "env_steps_per_epoch": steps / a.steps,
                              "avg_ep_ret": m1.get("AverageEpRet"),
                              **({"rollout_s_per_epoch": (m1["RolloutS"] - m0["RolloutS"]) / a.steps,
                                  "learn_s_per_epoch": (m1["LearnS"] - m0["LearnS"]) / a.steps,
                                  "overlap": bool(getattr(tr, "overlap", False))} if "RolloutS" in m1 else {}),
                              # C++ host rollout loop, per env step (driver thread wall time)
                              **{k: round(v, 2) for k, v in m1.items() if k.startswith("Host") and k.endswith("Us")}}),
                  flush=True)
        if hasattr(tr, "close"):
            tr.close()
        del tr
        if dev.type == "cuda":
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
