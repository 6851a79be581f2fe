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
    h.rollout(0, params, H, state, ep_len, ep_ret, obs, act, logp, rew, done, None, stats, seed, step0, True, max_steps)
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
        h.rollout(env, params, H, bufs["state"], bufs["ep_len"], bufs["ep_ret"], obs, act, f[0], f[1], f[2], None,
                  stats, 1, 0, True, ms)
        torch.cuda.synchronize()
        assert torch.isfinite(obs).all()
        assert int(act.max().item()) < A and int(act.min().item()) >= 0


def _lander_step_np(o, a, noise01):
    """numpy float32 oracle of LunarLanderSynthEnv.step (csrc/kernels/envs.h) from the obs."""
    f = np.float32
    x, y, vx, vy, ang, angv = (o[:, i].astype(f) for i in range(6))

    def shaping(x, y, vx, vy, ang):
        return (-100 * np.sqrt(x * x + y * y) - 100 * np.sqrt(vx * vx + vy * vy) - 100 * np.abs(ang)
                + np.where(y < 0.05, f(20), f(0))).astype(f)

    prev = shaping(x, y, vx, vy, ang)
    dt = f(1 / 50)
    main = a == 2
    side = (a == 1) | (a == 3)
    d = np.where(a == 1, f(-1), f(1))
    ax = np.where(main, -np.sin(ang) * f(13 / 6), np.where(side, d * np.cos(ang) * f(0.6 / 6), f(0)))
    ay = f(-10 / 6) + np.where(main, np.cos(ang) * f(13 / 6), f(0))
    aa = np.where(side, -d * f(1.5), f(0))
    fuel = np.where(main, f(0.3), np.where(side, f(0.03), f(0)))
    ax = ax + f(-0.05) + f(0.1) * noise01
    vx = vx + ax * dt * f(6)
    vy = vy + ay * dt * f(6)
    angv = angv + aa * dt
    x = x + vx * dt
    y = y + vy * dt
    ang = ang + angv * dt
    sh = shaping(x, y, vx, vy, ang)
    rew = sh - prev - fuel
    return np.stack([x, y, vx, vy, ang, angv], 1), rew


def test_lunarlander_device_rollout_matches_oracle(cuda):
    h = hip()
    env = 3
    D, A, NS, ms = h.env_dims(env)
    assert (D, A, ms) == (8, 4, 1000)
    N, T, H, seed = 256, 40, 128, 5
    params = MLPSpec(D, H, A).init(torch.Generator().manual_seed(3)).to(cuda)
    state = torch.zeros(N, NS, device=cuda)
    ep_len = torch.zeros(N, dtype=torch.int32, device=cuda)
    ep_ret = torch.zeros(N, device=cuda)
    obs = torch.zeros(T + 1, N, D, device=cuda)
    act = torch.zeros(T, N, dtype=torch.int32, device=cuda)
    logp, rew, done = (torch.zeros(T, N, device=cuda) for _ in range(3))
    stats = torch.zeros(h.rollout_grid(N), 8, device=cuda)
    h.rollout(env, params, H, state, ep_len, ep_ret, obs, act, logp, rew, done, None, stats, seed, 0, True, ms)
    torch.cuda.synchronize()
    o, a, r, d = obs.cpu().numpy(), act.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
    checked = 0
    for t in range(T):
        u = philox.uniforms(seed, t, np.arange(N), 0)
        ns, rr = _lander_step_np(o[t], a[t], u[1])
        live = d[t] == 0
        np.testing.assert_allclose(o[t + 1][live, :6], ns[live], rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(r[t][live], rr[live], rtol=1e-3, atol=1e-3)
        checked += live.sum()
    assert checked > N * T // 2
    assert np.isin(np.unique(a), np.arange(4)).all()


def test_halfcheetah_gaussian_device_rollout_matches_oracle(cuda):
    """Continuous fused rollout: Gaussian actions / log-probs vs the fp32 MLP oracle and the
    env transition vs a numpy oracle of HalfCheetahSynth with the kernel's Philox noise."""
    from relayrl_prototype_amd import _native

    h = hip()
    env = 4
    D, A, NS, ms = h.env_dims(env)
    assert (D, A) == (17, 6)
    N, T, H, seed = 128, 6, 128, 11
    spec = MLPSpec(D, H, A, gaussian=True)
    params = spec.init(torch.Generator().manual_seed(2))
    cst = np.asarray(_native.env_constants("HalfCheetahSynth-v0"), np.float32)
    Am, Bm = cst[:289].reshape(17, 17), cst[289:].reshape(17, 6)
    state = torch.zeros(N, NS, device=cuda)
    ep_len = torch.zeros(N, dtype=torch.int32, device=cuda)
    ep_ret = torch.zeros(N, device=cuda)
    obs = torch.zeros(T + 1, N, D, device=cuda)
    act = torch.zeros(T, N, A, device=cuda)
    logp, rew, done = (torch.zeros(T, N, device=cuda) for _ in range(3))
    stats = torch.zeros(h.rollout_grid(N), 8, device=cuda)
    h.rollout_cont(env, params.to(cuda), torch.from_numpy(cst).to(cuda), H, state, ep_len, ep_ret, obs, act, logp,
                   rew, done, None, stats, seed, 0, True, ms)
    torch.cuda.synchronize()
    o, a, lp, r = obs.cpu(), act.cpu(), logp.cpu(), rew.cpu()
    ls = params[spec.offsets()["log_std"]:spec.offsets()["log_std"] + A]
    for t in range(T):
        mu = ref.mlp_forward_ref(3, params, o[t], A, H)["logits"]
        z = (a[t] - mu) / torch.exp(ls)
        lp_ref = (-0.5 * z * z - ls - 0.9189385332046727).sum(-1)
        torch.testing.assert_close(lp[t], lp_ref, rtol=1e-3, atol=2e-3)
        u = np.clip(a[t].numpy(), -1, 1)
        pre = o[t].numpy() @ Am.T + u @ Bm.T
        noise = np.concatenate([np.stack(philox.uniforms(seed, t, np.arange(N), 8 + q), 1) for q in range(5)], 1)
        ns = np.tanh(pre) + (-0.01 + 0.02 * noise[:, :17])
        np.testing.assert_allclose(o[t + 1].numpy(), ns, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(r[t].numpy(), ns[:, 8] - 0.1 * (u * u).sum(1), rtol=1e-4, atol=1e-4)
    # sampled actions are mu + std * N(0, 1)
    zs = ((a - torch.stack([ref.mlp_forward_ref(3, params, o[t], A, H)["logits"] for t in range(T)]))
          / torch.exp(ls)).reshape(-1)
    assert abs(zs.mean().item()) < 0.05 and abs(zs.std().item() - 1.0) < 0.05
