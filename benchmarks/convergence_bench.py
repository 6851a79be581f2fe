#!/usr/bin/env python3
"""Learning curves of the device presets at full speed: AverageEpRet against wall-clock
seconds and env steps, one JSON line per preset (rank 0).  Throughput benchmarks say how
fast an epoch runs; this says the same epochs learn (synthetic envs, random-init weights).

    python benchmarks/convergence_bench.py --presets halfcheetah-ppo lunarlander-reinforce-baseline \\
        --epochs 150
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(preset: str, epochs: int, every: int) -> dict:
    from relayrl_prototype_amd.runtime.launcher import run_preset

    curve = []
    t0 = time.perf_counter()

    def on_metrics(m):
        if int(m.get("Epoch", 0)) % every == 0 or not curve:
            curve.append({"epoch": int(m.get("Epoch", 0)), "s": round(time.perf_counter() - t0, 3),
                          "env_steps": int(m.get("EnvSteps", 0)), "avg_ep_ret": m.get("AverageEpRet"),
                          "ep_len": m.get("EpLen")})

    with tempfile.TemporaryDirectory() as out:
        last = run_preset(preset, epochs, out, {}, on_metrics=on_metrics)
    rets = [c["avg_ep_ret"] for c in curve if c["avg_ep_ret"] == c["avg_ep_ret"]]
    return {"preset": preset, "epochs": epochs, "wall_s": round(time.perf_counter() - t0, 2),
            "env_steps": int(last.get("EnvSteps", 0)), "first_avg_ep_ret": rets[0] if rets else None,
            "best_avg_ep_ret": max(rets) if rets else None, "last_avg_ep_ret": rets[-1] if rets else None,
            "curve": curve, "data": "synthetic device envs, random-init weights"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--presets", nargs="+", default=["cartpole-reinforce-baseline", "lunarlander-reinforce-baseline",
                                                     "halfcheetah-ppo"])
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--every", type=int, default=5, help="curve resolution (epochs)")
    a = ap.parse_args()
    for p in a.presets:
        print(json.dumps(run(p, a.epochs, a.every)), flush=True)


if __name__ == "__main__":
    main()
