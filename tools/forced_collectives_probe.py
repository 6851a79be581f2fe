#!/usr/bin/env python3
"""The world > 1 optimiser path on ONE GPU: a one-rank RCCL group forced through the
multi-rank code (``RRL_FORCE_COLLECTIVES=1`` -> ``Comm.multi``): slab reduce -> real
``dist.all_reduce`` -> Adam per optimiser step, the Pong DP update's bucketed all-reduces.

* ``--check``: captured (hipGraph, RCCL all-reduces inside) vs eager must be BITWISE equal
  after a few epochs -- CartPole REINFORCE-with-baseline (whole optimize() epoch captured)
  and the Pong A2C update.  Also asserts the multi path really ran (``comm.multi``, nccl,
  graph replays counted).
* ``--bench``: the LunarLander preset epoch (2048 envs x 128 steps, 80 value iterations)
  eager vs captured on the forced path, and captured at plain world 1, so the per-iteration
  cost the multi-rank path adds over world 1 is measured, not modelled.

Prints one JSON line.  Run in its own process (it owns the process group).
"""
import argparse
import json
import os
import sys
import time

os.environ["RRL_FORCE_COLLECTIVES"] = "1"
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from relayrl_prototype_amd.parallel.comm import Comm, init_distributed  # noqa: E402


def _vec(comm, graphs, env="CartPole-v1", n=2048, t=16, vi=8, seed=3):
    from relayrl_prototype_amd.runtime.vec_trainer import VecTrainer, VecTrainerConfig

    cfg = VecTrainerConfig(env=env, num_envs=n, rollout_len=t, train_vf_iters=vi, use_graphs=graphs, seed=seed)
    return VecTrainer(cfg, comm)


def check(comm) -> dict:
    out = {}
    res = {}
    for graphs in (False, True):
        tr = _vec(comm, graphs)
        for _ in range(4):
            tr.train_epoch()
        torch.cuda.synchronize()
        res[graphs] = (tr.pi.params.clone(), tr.vf.params.clone(), tr.learner.graph_replays, tr.pi.version,
                       tr.vf.version)
    e, g = res[False], res[True]
    out["vec_pi_bitwise"] = bool(torch.equal(e[0], g[0]))
    out["vec_vf_bitwise"] = bool(torch.equal(e[1], g[1]))
    out["vec_graph_replays"] = int(g[2])
    out["vec_eager_replays"] = int(e[2])
    out["vec_versions_equal"] = (e[3], e[4]) == (g[3], g[4])
    from relayrl_prototype_amd.runtime.pixel_trainer import PixelA2CConfig, PixelA2CTrainer

    pres = {}
    for graphs in (False, True):
        tr = PixelA2CTrainer(PixelA2CConfig(num_envs=256, rollout_len=5, seed=2, use_graphs=graphs), comm=comm)
        for _ in range(4):
            tr.train_epoch()
        torch.cuda.synchronize()
        pres[graphs] = (tr.model.params.clone(), len(tr._graphs))
        del tr
    out["pong_params_bitwise"] = bool(torch.equal(pres[False][0], pres[True][0]))
    out["pong_graphs"] = pres[True][1]
    out["pong_eager_graphs"] = pres[False][1]
    return out


def bench(comm, plain, epochs: int, warmup: int) -> dict:
    rec = {}
    for name, c, graphs in (("forced_eager", comm, False), ("forced_graph", comm, True), ("world1_graph", plain, True),
                            ("world1_eager", plain, False)):
        tr = _vec(c, graphs, env="LunarLanderSynth-v0", n=2048, t=128, vi=80, seed=1)
        for _ in range(warmup):
            tr.train_epoch()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(epochs):
            tr.train_epoch()
        torch.cuda.synchronize()
        rec[name + "_ms_per_epoch"] = round((time.perf_counter() - t0) / epochs * 1e3, 3)
        rec[name + "_replays"] = tr.learner.graph_replays
        del tr
        torch.cuda.empty_cache()
    it = 81  # 1 policy step + 80 value steps per epoch
    rec["multi_path_overhead_us_per_iter_graph"] = round(
        (rec["forced_graph_ms_per_epoch"] - rec["world1_graph_ms_per_epoch"]) * 1e3 / it, 2)
    rec["multi_path_overhead_us_per_iter_eager"] = round(
        (rec["forced_eager_ms_per_epoch"] - rec["world1_graph_ms_per_epoch"]) * 1e3 / it, 2)
    rec["capture_saves_us_per_iter"] = round(
        (rec["forced_eager_ms_per_epoch"] - rec["forced_graph_ms_per_epoch"]) * 1e3 / it, 2)
    rec["config"] = "LunarLanderSynth-v0 REINFORCE-with-baseline, 2048 envs x 128 steps, 80 value iterations"
    return rec


def syncs(comm, plain, epochs: int) -> dict:
    """the multi-rank engine loop (EngineRunner with the stop agreement of a
    relay-attached rank 0, ``log_every=0``) on the forced path: synchronising host reads per
    steady-state epoch (Tensor.item / tolist / cpu, torch.cuda.synchronize), counted by hooks,
    and the epoch time against the world-1 graph path."""
    import tempfile
    from collections import Counter

    from relayrl_prototype_amd.runtime.engine import EngineAlgorithm, EngineRunner, EngineSpec

    counts = Counter()
    active = [False]
    orig = {"item": torch.Tensor.item, "tolist": torch.Tensor.tolist, "cpu": torch.Tensor.cpu,
            "synchronize": torch.cuda.synchronize, "event_wait": torch.cuda.Event.synchronize}

    def hook(name, fn):
        def w(*a, **k):
            if active[0]:
                counts[name] += 1
            return fn(*a, **k)
        return w

    torch.Tensor.item = hook("item", orig["item"])
    torch.Tensor.tolist = hook("tolist", orig["tolist"])
    torch.Tensor.cpu = hook("cpu", orig["cpu"])
    torch.cuda.synchronize = hook("synchronize", orig["synchronize"])
    torch.cuda.Event.synchronize = hook("event_wait", orig["event_wait"])

    class _Pub:
        updates = 0

        def publish_model(self):
            pass

    rec = {}
    try:
        for name, c, agree in (("forced_relay", comm, True), ("world1", plain, False)):
            spec = EngineSpec("vec", "LunarLanderSynth-v0", "reinforce", 1,
                              {"env": "LunarLanderSynth-v0", "algo": "reinforce", "num_envs": 2048, "rollout_len": 128,
                               "train_vf_iters": 80, "seed": 1, "use_graphs": True})
            algo = EngineAlgorithm(spec, tempfile.mkdtemp(), comm=c, device=torch.device("cuda", 0), log=False)
            r = EngineRunner(algo, _Pub(), time.perf_counter())
            r.agree_stop = agree
            r.train(epochs=4, log_every=0, publish_every=0)  # warm-up + captures
            orig["synchronize"]()
            counts.clear()
            active[0] = True
            t0 = time.perf_counter()
            r.train(epochs=epochs, log_every=0, publish_every=0)
            active[0] = False
            orig["synchronize"]()
            el = time.perf_counter() - t0
            rec[name + "_ms_per_epoch"] = round(el / epochs * 1e3, 3)
            rec[name + "_sync_reads_per_epoch"] = round(sum(v for k, v in counts.items() if k != "event_wait") / epochs, 3)
            rec[name + "_lagged_event_waits_per_epoch"] = round(counts["event_wait"] / epochs, 3)
            rec[name + "_hooks"] = dict(counts)
            del r, algo
            torch.cuda.empty_cache()
    finally:
        torch.Tensor.item, torch.Tensor.tolist, torch.Tensor.cpu = orig["item"], orig["tolist"], orig["cpu"]
        torch.cuda.synchronize, torch.cuda.Event.synchronize = orig["synchronize"], orig["event_wait"]
    rec["relay_overhead_pct"] = round((rec["forced_relay_ms_per_epoch"] / rec["world1_ms_per_epoch"] - 1) * 100, 2)
    rec["syncs_config"] = "LunarLanderSynth-v0 REINFORCE-with-baseline, 2048 envs x 128 steps, 80 value iterations"
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--bench", action="store_true")
    ap.add_argument("--syncs", action="store_true")
    ap.add_argument("--epochs", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    comm = init_distributed()
    out = {"backend": comm.backend, "world": comm.world, "multi": comm.multi, "graph_safe": comm.graph_safe}
    assert comm.multi and comm.backend == "nccl", out
    if a.check:
        out.update(check(comm))
    if a.bench:
        out.update(bench(comm, Comm(collectives=False), a.epochs, a.warmup))
    if a.syncs:
        out.update(syncs(comm, Comm(collectives=False), max(a.epochs, 20)))
    import torch.distributed as dist

    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
