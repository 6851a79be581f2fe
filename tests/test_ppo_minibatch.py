"""PPO shuffled-minibatch schedule (algorithms/learner.py num_minibatches).

Oracle: M minibatch steps per epoch equal M full-batch optimize() calls, one per minibatch
of the same permutation, each normalising by its own row count.  The reference ships no
PPO (config_loader.rs:398-399 only whitelists the name), so parity is unpinned; this pins
the schedule against the single-step path that the kernel oracles already cover.
"""
import pytest
import torch

from relayrl_prototype_amd.algorithms.learner import PGLearner
from relayrl_prototype_amd.ops import FwdMode, mlp_forward, scan_flat


def _batch(B, D, A, discrete, device, seed=0):
    g = torch.Generator().manual_seed(seed)
    obs = torch.randn(B, D, generator=g)
    rew = torch.randn(B, generator=g)
    done = (torch.rand(B, generator=g) < 0.05).float()
    done[-1] = 1.0
    val = torch.randn(B, generator=g) * 0.1
    boot = torch.zeros(B)
    if discrete:
        act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32)
        actc = None
    else:
        act = None
        actc = torch.randn(B, A, generator=g)
    to = lambda t: None if t is None else t.to(device)
    obs, rew, done, val, boot, act, actc = map(to, (obs, rew, done, val, boot, act, actc))
    adv, ret, stats = scan_flat(rew, done, val, boot, 0.99, 0.95)
    return obs, act, actc, adv, ret, stats


def _learner(discrete, D, A, device, M, pi_iters, vf_iters, seed=3):
    return PGLearner("ppo", D, A, 128, discrete, True, 3e-3, 1e-3, vf_iters, pi_iters, device=device, seed=seed,
                     use_graphs=False, num_minibatches=M)


def _check(device, discrete, B=1000, M=4, pi_iters=2, vf_iters=2, D=6, A=3):
    obs, act, actc, adv, ret, stats = _batch(B, D, A, discrete, device)
    mode = FwdMode.CAT_EVAL if discrete else FwdMode.GAUSS_EVAL
    mb = _learner(discrete, D, A, device, M, pi_iters, vf_iters)
    logp_old = mlp_forward(mode, mb.pi.params, obs, A, 128, act_in=act, actc_in=actc)["logp"].detach()
    mb.optimize(obs, act=act, actc=actc, adv=adv, ret=ret, adv_stats=stats, logp_old=logp_old)

    ref = _learner(discrete, D, A, device, 1, 1, 1)
    gen = torch.Generator(device=device).manual_seed(mb.mb_seed)
    sel = lambda t, idx: None if t is None else t.index_select(0, idx)

    def perms():
        p = torch.randperm(B, device=device, generator=gen)
        return [p[i * B // M:(i + 1) * B // M] for i in range(M)]

    ref.train_vf_iters = 0
    for _ in range(pi_iters):
        for idx in perms():
            ref.optimize(sel(obs, idx), act=sel(act, idx), actc=sel(actc, idx), adv=sel(adv, idx), ret=sel(ret, idx),
                         adv_stats=stats, logp_old=sel(logp_old, idx), inv_B=1.0 / idx.numel())
    ref.train_pi_iters, ref.train_vf_iters = 0, 1
    for _ in range(vf_iters):
        for idx in perms():
            ref.optimize(sel(obs, idx), ret=sel(ret, idx), adv_stats=stats, inv_B=1.0 / idx.numel())
    assert mb.pi.version == ref.pi.version == pi_iters * M
    assert mb.vf.version == ref.vf.version == vf_iters * M
    torch.testing.assert_close(mb.pi.params, ref.pi.params, rtol=0, atol=0)
    torch.testing.assert_close(mb.vf.params, ref.vf.params, rtol=0, atol=0)
    s = mb.summarize()
    assert all(map(lambda k: s[k] == s[k], ("LossPi", "LossV", "KL")))


@pytest.mark.parametrize("discrete", [True, False])
def test_ppo_minibatch_schedule_cpu(discrete):
    _check("cpu", discrete)


def test_ppo_minibatch_kl_stop_cpu():
    """Early stopping checks the KL of every minibatch step after the first and ends the epoch loop."""
    obs, act, actc, adv, ret, stats = _batch(2048, 6, 3, True, "cpu", seed=1)
    lr = PGLearner("ppo", 6, 3, 128, True, True, 5e-2, 1e-3, 0, 20, target_kl=1e-4, device="cpu", seed=0,
                   use_graphs=False, num_minibatches=8)
    logp_old = mlp_forward(FwdMode.CAT_EVAL, lr.pi.params, obs, 3, 128, act_in=act)["logp"].detach()
    lr.optimize(obs, act=act, adv=adv, ret=ret, adv_stats=stats, logp_old=logp_old)
    assert lr.last["kl_stop"] is not None and lr.pi.version < 20 * 8


def test_minibatch_config_plumbing():
    from relayrl_prototype_amd.runtime.host_trainer import HostTrainerConfig, HostVecTrainer

    tr = HostVecTrainer(HostTrainerConfig(env="CartPole-v1", num_envs=64, rollout_len=16, algo="ppo",
                                          train_pi_iters=2, train_vf_iters=2, num_minibatches=4, num_threads=2),
                        device="cpu")
    tr.train_epoch()
    assert tr.learner.num_minibatches == 4 and tr.learner.pi.version == 8 and tr.learner.vf.version == 8


@pytest.mark.gpu
@pytest.mark.parametrize("discrete", [True, False])
def test_ppo_minibatch_schedule_gpu(cuda, discrete):
    _check(cuda, discrete, B=4096, D=4 if discrete else 17, A=3 if discrete else 6)
