"""BASELINE configs #3-#5 LEARN on the device engines (not only run fast): each preset must
lift the mean return of its newest >= 100 finished episodes past a bar within an epoch cap
(benchmarks/convergence_bench.py; the full thresholds and wall-clock are in bench.py's
``convergence`` block and profiles/r5_convergence*.jsonl).

The bars are cheaper than the bench thresholds and leave a margin over the epochs seed 1
needed on an MI355X (Pong: -20 -> -15 by update 784 of 2,048 envs x 5 steps; LunarLander: 0
by epoch 248; HalfCheetah: 500 by epoch 184).  The reference's own evidence of this kind is
the LunarLander notebook's logged learning run (lunar_lander_zmq.ipynb, REINFORCE.py:97-125).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(name, cap, budget=90.0, seed=1, **ov):
    from benchmarks.convergence_bench import run

    return run(name, ov, cap, budget, 100, seed)


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_pong_a2c_learns_to_return_the_ball():
    r = _run("pong-a2c", cap=1600)
    first = next(c["window_ret"] for c in r["curve"] if c["window_ret"] is not None)
    assert r["thresholds"]["-15.0"] is not None, r["curve"]
    assert r["best_window_ret"] >= first + 5.0, (first, r["best_window_ret"])


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_lunarlander_reinforce_baseline_reaches_zero():
    r = _run("lunarlander-reinforce-baseline", cap=450)
    assert r["thresholds"]["0.0"] is not None, r["curve"]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_halfcheetah_ppo_climbs_past_450():
    r = _run("halfcheetah-ppo", cap=260)
    assert r["thresholds"]["450.0"] is not None, r["curve"]
