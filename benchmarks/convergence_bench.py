#!/usr/bin/env python3
"""Time-to-threshold of the BASELINE.json learning configs (#2-#5) on the device engines:
the mean return of the newest >= ``window`` finished episodes (vec_trainer.SolvedCheck, the
gymnasium criterion) against wall-clock seconds and env steps, with fixed seeds.

The reference's runs are learning runs (the LunarLander ZMQ notebook logs 102 AverageEpRet
rows of REINFORCE.py:97-125); throughput benchmarks only say how fast an epoch runs, this
says the same epochs learn.  Synthetic envs (docs/ENVS.md), random-init weights.

    python benchmarks/convergence_bench.py --presets pong-a2c lunarlander-reinforce-baseline halfcheetah-ppo
    python benchmarks/convergence_bench.py --presets pong-a2c --set lr=5e-4 --max-seconds 60

One JSON line per preset (rank 0): the wall-clock and env steps at which each threshold was
first reached, and the curve (window return every ``--every`` epochs).  The clock starts
before the trainer is built (allocation + first-epoch warm-up / graph capture included) and
stops when the solved epoch's episode sums reach the host; the per-epoch check is one
synchronising read of two sums.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# name -> launcher preset, overrides, thresholds (ascending), window, wall-clock budget (s)
CONV = {
    "cartpole-reinforce-baseline": dict(
        preset="cartpole-reinforce-baseline", overrides={"num_envs": 512, "rollout_len": 16},
        thresholds=[200.0, 475.0], window=100, budget=60.0,
        note="reference hyperparameters (gamma .98, lam .97, pi_lr 3e-4, vf_lr 1e-3, 80 value iterations)"),
    "lunarlander-reinforce-baseline": dict(
        preset="lunarlander-reinforce-baseline", overrides={},
        thresholds=[0.0, 100.0], window=100, budget=120.0,
        note="LunarLanderSynth-v0 (point-mass lander, gymnasium shaping, +-100 terminal bonus)"),
    "halfcheetah-ppo": dict(
        preset="halfcheetah-ppo", overrides={"num_minibatches": 16},
        thresholds=[450.0, 500.0, 550.0], window=100, budget=120.0,
        note="HalfCheetahSynth-v0 (s' = tanh(A s + B u) + noise, reward s'[8] - 0.1|u|^2, 1000 steps); 16 shuffled "
             "minibatches per PPO epoch (the preset's full-batch schedule reaches 500 at ~9 s, plateaus ~563)"),
    "pong-a2c": dict(
        preset="pong-a2c", overrides={"num_envs": 2048},
        thresholds=[-15.0, -5.0, 0.0, 10.0, 15.0, 19.0], window=100, budget=150.0,
        note="PongSynth-v0 vs the tracking opponent; 0 = wins as many points as it loses"),
}


def episode_sums(tr):
    return tr.episode_sums()


def run(name: str, overrides: dict, epochs: int, max_seconds: float, every: int, seed: int) -> dict:
    import torch

    from relayrl_prototype_amd.parallel.comm import Comm
    from relayrl_prototype_amd.runtime.launcher import PRESETS, _epoch, _make_trainer
    from relayrl_prototype_amd.runtime.vec_trainer import SolvedCheck

    c = CONV[name]
    ov = dict(c["overrides"])
    ov["seed"] = seed
    ov.update(overrides)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr = _make_trainer(PRESETS[c["preset"]], Comm(), dev, ov)
    checks = [SolvedCheck(th, c["window"]) for th in c["thresholds"]]
    hit = {}
    curve = []
    budget = max_seconds if max_seconds else c["budget"]
    ep = 0
    steps_per_epoch = None
    last_win = float("nan")
    best = float("-inf")
    t_print = t0
    while True:
        _epoch(tr)
        ep += 1
        n, s = episode_sums(tr)
        el = time.perf_counter() - t0
        env_steps = int(getattr(tr, "env_steps", 0) or getattr(tr, "total_steps", 0))
        if steps_per_epoch is None:
            steps_per_epoch = env_steps
        win = float("nan")
        for th, ck in zip(c["thresholds"], checks):
            win = ck.update(n, s)
            if th not in hit and ck.solved(win):
                hit[th] = {"s": round(el, 3), "env_steps": env_steps, "epoch": ep}
        last_win = win
        if win == win:
            best = max(best, win)
        if ep % every == 0 or ep == 1:
            curve.append({"epoch": ep, "s": round(el, 3), "env_steps": env_steps,
                          "window_ret": None if win != win else round(win, 3), "episodes": n})
        if el - (t_print - t0) >= 15.0:  # progress for long runs (stderr)
            t_print = time.perf_counter()
            print(f"[{name}] epoch {ep} {el:.1f}s steps {env_steps} window {win:.2f} hit {sorted(hit)}",
                  file=sys.stderr, flush=True)
        if len(hit) == len(checks) or el >= budget or (epochs and ep >= epochs):
            break
    if dev.type == "cuda":
        torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    m = tr.metrics() if hasattr(tr, "metrics") else {}
    if hasattr(tr, "close"):
        tr.close()
    return {"preset": name, "seed": seed, "overrides": ov, "note": c["note"], "window": c["window"],
            "thresholds": {str(th): hit.get(th) for th in c["thresholds"]},
            "solved_all": len(hit) == len(checks), "epochs": ep, "wall_s": round(wall, 2),
            "env_steps": int(getattr(tr, "env_steps", 0) or getattr(tr, "total_steps", 0)),
            "env_steps_per_epoch": steps_per_epoch, "last_window_ret": None if last_win != last_win else last_win,
            "best_window_ret": None if best == float("-inf") else best,
            "entropy": m.get("Entropy"), "curve": curve,
            "data": "synthetic device envs, random-init weights"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--presets", nargs="+", default=["pong-a2c", "lunarlander-reinforce-baseline", "halfcheetah-ppo"])
    ap.add_argument("--epochs", type=int, default=0, help="epoch cap (0: until solved or the budget)")
    ap.add_argument("--max-seconds", type=float, default=0.0, help="wall-clock budget per run (0: the preset's)")
    ap.add_argument("--every", type=int, default=10, help="curve resolution (epochs)")
    ap.add_argument("--seeds", type=int, nargs="+", default=[1])
    ap.add_argument("--set", nargs="*", default=[], help="trainer overrides key=value")
    ap.add_argument("--out", default=None, help="append the JSON lines to this file too")
    a = ap.parse_args()
    ov = {}
    for kv in a.set:
        k, v = kv.split("=", 1)
        try:
            v = json.loads(v)
        except ValueError:
            pass
        ov[k] = v
    for p in a.presets:
        for s in a.seeds:
            line = json.dumps(run(p, ov, a.epochs, a.max_seconds, a.every, s))
            print(line, flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(line + "\n")


if __name__ == "__main__":
    main()
