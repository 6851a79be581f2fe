"""Fused on-device rollout kernel vs a host re-simulation (physics + Philox + policy oracle)."""
import numpy as np
import pytest
import torch

from relayrl_prototype_amd.ops import MLPSpec, hip
from relayrl_prototype_amd.ops import reference as ref
from relayrl_prototype_amd.ops import philox

pytestmark = pytest.mark.gpu


def cartpole_step_np(s, a):
    s = s.astype(np.float32)
    x, xd, th, thd = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
    force = np.where(a == 1, np.float32(10.0), np.float32(-10.0))
    costh, sinth = np.cos(th), np.sin(th)
    temp = (force + np.float32(0.05) * thd * thd * sinth) / np.float32(1.1)
    thacc = (np.float32(9.8) * sinth - costh * temp) / (
        np.float32(0.5) * (np.float32(4.0 / 3.0) - np.float32(0.1) * costh * costh / np.float32(1.1)))
    xacc = temp - np.float32(0.05) * thacc * costh / np.float32(1.1)
    ns = np.stack([x + 0.02 * xd, xd + 0.02 * xacc, th + 0.02 * thd, thd + 0.02 * thacc], 1).astype(np.float32)
    lim = 12 * 2 * np.pi / 360
    term = (ns[:, 0] < -2.4) | (ns[:, 0] > 2.4) | (ns[:, 2] < -lim) | (ns[:, 2] > lim)
    return ns, term


@pytest.mark.parametrize("N,T,H", [(100, 40, 128), (37, 600, 64)])
def test_cartpole_rollout(cuda, N, T, H):
    h = hip()
    D, A, NS, max_steps = h.env_dims(0)
    assert (D, A, NS, max_steps) == (4, 2, 4, 500)
    spec = MLPSpec(D, H, A)
    params = spec.init(torch.Generator().manual_seed(3)).to(cuda)
    dev = cuda
    state = torch.zeros(N, NS, device=dev)
    ep_len = torch.zeros(N, dtype=torch.int32, device=dev)
    ep_ret = torch.zeros(N, device=dev)
    obs = torch.zeros(T + 1, N, D, device=dev)
    act = torch.zeros(T, N, dtype=torch.int32, device=dev)
    logp = torch.zeros(T, N, device=dev)
    rew = torch.zeros(T, N, device=dev)
    done = torch.zeros(T, N, device=dev)
    stats = torch.zeros(h.rollout_grid(N), 8, device=dev)
    seed, step0 = 777, 1000
    h.rollout(0, params, H, state, ep_len, ep_ret, obs, act, logp, rew, done, stats, seed, step0, True, max_steps)
    torch.cuda.synchronize()
    obs_c, act_c, logp_c, done_c = obs.cpu(), act.cpu(), logp.cpu(), done.cpu()
    # initial reset state from Philox tag 1
    u = philox.uniforms(seed, step0, np.arange(N), 1)
    s0 = np.stack([-0.05 + 0.1 * x for x in u], 1).astype(np.float32)
    np.testing.assert_allclose(obs_c[0].numpy(), s0, rtol=0, atol=1e-6)
    # log-probs are log_softmax of the policy at the stored observation
    pc = params.cpu()
    for t in range(0, T, max(1, T // 7)):
        r = ref.mlp_forward_ref(2, pc, obs_c[t], A, H, act_in=act_c[t])
        torch.testing.assert_close(logp_c[t], r["logp"], rtol=1e-4, atol=1e-4)
        rs = ref.mlp_forward_ref(1, pc, obs_c[t], A, H, seed=seed, step=step0 + t)
        assert (rs["act"] != act_c[t]).float().mean().item() <= 0.02
    # physics: non-terminal transitions follow the Euler update
    ok = 0
    for t in range(T - 1):
        ns, term = cartpole_step_np(obs_c[t].numpy(), act_c[t].numpy())
        nd = done_c[t].numpy() == 0
        np.testing.assert_allclose(obs_c[t + 1].numpy()[nd], ns[nd], rtol=1e-4, atol=1e-5)
        # a done step is either a physics termination or the 500-step time limit
        d = done_c[t].numpy() > 0
        assert np.all(term[d] | (T > 500)), t
        ok += nd.sum()
    assert ok > 0
    assert torch.all(rew.cpu() == 1.0)
    st = stats.sum(0).cpu()
    assert int(st[0].item()) == int(done_c.sum().item())


def test_rollout_other_envs(cuda):
    h = hip()
    for env in (1, 2):
        D, A, NS, ms = h.env_dims(env)
        N, T, H = 64, 50, 128
        params = MLPSpec(D, H, A).init(torch.Generator().manual_seed(env)).to(cuda)
        bufs = dict(state=torch.zeros(N, NS, device=cuda), ep_len=torch.zeros(N, dtype=torch.int32, device=cuda),
                    ep_ret=torch.zeros(N, device=cuda))
        obs = torch.zeros(T + 1, N, D, device=cuda)
        act = torch.zeros(T, N, dtype=torch.int32, device=cuda)
        f = [torch.zeros(T, N, device=cuda) for _ in range(3)]
        stats = torch.zeros(h.rollout_grid(N), 8, device=cuda)
        h.rollout(env, params, H, bufs["state"], bufs["ep_len"], bufs["ep_ret"], obs, act, f[0], f[1], f[2], stats,
                  1, 0, True, ms)
        torch.cuda.synchronize()
        assert torch.isfinite(obs).all()
        assert int(act.max().item()) < A and int(act.min().item()) >= 0
