"""Host-env vectorised trainer on the CPU oracle path (the GPU path is in test_trainers_gpu.py)."""
import math

import pytest
import torch

from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer


@pytest.mark.parametrize("env,algo", [("CartPole-v1", "reinforce"), ("Pendulum-v1", "ppo"),
                                      ("LunarLanderSynth-v0", "a2c"), ("HalfCheetahSynth-v0", "ppo")])
def test_host_trainer_cpu(env, algo):
    torch.set_num_threads(2)
    cfg = HostTrainerConfig(env=env, num_envs=8, rollout_len=20, algo=algo, hidden=64, train_vf_iters=2,
                            train_pi_iters=2, num_threads=2, seed=1)
    tr = HostVecTrainer(cfg, device="cpu")
    p0 = tr.learner.pi.params.clone()
    for _ in range(2):
        tr.train_epoch()
    m = tr.metrics()
    assert m["EnvSteps"] == 2 * 8 * 20
    assert math.isfinite(m["LossPi"]) and math.isfinite(m["LossV"])
    assert not torch.equal(p0, tr.learner.pi.params)


def test_cartpole_reinforce_learns_cpu():
    """Convergence smoke (SURVEY §4 e): CartPole average return rises well above random (~22)."""
    torch.manual_seed(0)
    torch.set_num_threads(4)
    cfg = HostTrainerConfig(env="CartPole-v1", num_envs=32, rollout_len=100, algo="ppo", hidden=64, pi_lr=3e-3,
                            vf_lr=3e-3, train_vf_iters=10, train_pi_iters=10, num_threads=2, seed=0, gamma=0.99)
    tr = HostVecTrainer(cfg, device="cpu")
    best = 0.0
    for _ in range(25):
        tr.train_epoch()
        m = tr.metrics()
        if m["Episodes"]:
            best = max(best, m["AverageEpRet"])
        if best > 100:
            break
    assert best > 100, best


def test_actor_learner_single_rank_colocated():
    """One rank that both acts and learns (the 1-GPU form of BASELINE config 3)."""
    from relayrl_prototype_amd.runtime.actor_learner import ActorLearner, ActorLearnerConfig

    al = ActorLearner(ActorLearnerConfig(env="LunarLanderSynth-v0", num_envs=8, rollout_len=16, learner_acts=True,
                                         hidden=64, train_vf_iters=2, num_threads=1), device="cpu")
    p0 = al.learner.pi.params.clone()
    for _ in range(2):
        al.step()
    al.finish()
    m = al.metrics()
    assert m["EnvSteps"] == 2 * 16 * 8 and not torch.equal(p0, al.learner.pi.params)
