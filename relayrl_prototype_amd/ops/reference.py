"""Pure-PyTorch fp32 oracles of every HIP kernel.

These are the numerics ground truth for the kernel tests (tests/test_kernels_gpu.py)
and the execution path for CPU tensors.  They implement the reference's math
(REINFORCE.py:141-160, kernel.py:23-37, replay_buffer.py:48-111,
BaseReplayBuffer.py:12-53) with the documented fixes: true log_softmax log-probs,
true entropy, and an epsilon in the advantage normalisation.
"""
from __future__ import annotations

import numpy as np
import torch

from . import philox

MODE_VALUE, MODE_CAT_SAMPLE, MODE_CAT_EVAL, MODE_LOGITS, MODE_GAUSS_SAMPLE, MODE_GAUSS_EVAL = range(6)
HEAD_PG_CAT, HEAD_VALUE_MSE, HEAD_PPO_CAT, HEAD_PPO_GAUSS, HEAD_PG_GAUSS = range(5)
HALF_LOG_2PI = 0.91893853320467274


def unflatten(params: torch.Tensor, D: int, H: int, A: int, gaussian: bool = False):
    o = 0

    def take(n, shape):
        nonlocal o
        t = params[o : o + n].view(*shape)
        o += n
        return t

    W1 = take(H * D, (H, D))
    b1 = take(H, (H,))
    W2 = take(H * H, (H, H))
    b2 = take(H, (H,))
    W3 = take(A * H, (A, H))
    b3 = take(A, (A,))
    log_std = take(A, (A,)) if gaussian else None
    return W1, b1, W2, b2, W3, b3, log_std


def trunk(params, X, D, H, A, gaussian=False):
    W1, b1, W2, b2, W3, b3, log_std = unflatten(params, D, H, A, gaussian)
    h1 = torch.relu(X @ W1.t() + b1)
    h2 = torch.relu(h1 @ W2.t() + b2)
    out = h2 @ W3.t() + b3
    return out, log_std


def masked_logits(logits, mask):
    if mask is None:
        return logits
    return logits + (mask - 1.0) * 1e8


def cat_sample_from_u(logits: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """Inverse-CDF draw matching rrl::cat_sample (first a with u < cdf[a] and p > 0)."""
    lse = torch.logsumexp(logits, dim=-1, keepdim=True)
    p = torch.exp(logits - lse)
    cdf = torch.cumsum(p, dim=-1)
    ok = (u.unsqueeze(-1) < cdf) & (p > 0)
    A = logits.shape[-1]
    idx = torch.arange(A, device=logits.device).expand_as(p)
    big = torch.full_like(idx, A)
    first = torch.where(ok, idx, big).min(dim=-1).values
    last_pos = torch.where(p > 0, idx, torch.full_like(idx, -1)).max(dim=-1).values
    return torch.where(first < A, first, last_pos.clamp(min=0))


@torch.no_grad()
def mlp_forward_ref(mode, params, X, A, H, mask=None, act_in=None, actc_in=None, seed=0, step=0, row_offset=0):
    B, D = X.shape
    gaussian = mode in (MODE_GAUSS_SAMPLE, MODE_GAUSS_EVAL)
    Aeff = 1 if mode == MODE_VALUE else A
    out, log_std = trunk(params.float(), X.float(), D, H, Aeff, gaussian)
    res = {}
    if mode == MODE_VALUE:
        res["v"] = out[:, 0]
        return res
    if not gaussian:
        logits = masked_logits(out, mask)
        logp_all = torch.log_softmax(logits, dim=-1)
        p = torch.exp(logp_all)
        ent = -(p * torch.where(p > 0, logp_all, torch.zeros_like(logp_all))).sum(-1)
        res["logits"] = logits
        res["entropy"] = ent
        if mode == MODE_CAT_SAMPLE:
            rows = np.arange(B, dtype=np.uint64) + np.uint64(row_offset)
            u = torch.from_numpy(philox.uniforms(seed, step, rows, 0)[0]).to(X.device)
            a = cat_sample_from_u(logits, u)
            res["act"] = a.to(torch.int32)
            res["logp"] = logp_all.gather(-1, a.long().unsqueeze(-1)).squeeze(-1)
        elif mode == MODE_CAT_EVAL:
            res["logp"] = logp_all.gather(-1, act_in.long().unsqueeze(-1)).squeeze(-1)
        return res
    mu = out
    std = torch.exp(log_std)
    if mode == MODE_GAUSS_SAMPLE:
        rows = np.arange(B, dtype=np.uint64) + np.uint64(row_offset)
        zs = []
        for a in range(A):
            u = philox.uniforms(seed, step, rows, 16 + (a & ~1))
            u1 = np.maximum(u[2] if a & 1 else u[0], np.float32(1e-7))
            u2 = u[3] if a & 1 else u[1]
            zs.append(np.sqrt(-2.0 * np.log(u1)) * np.cos(2 * np.pi * u2))
        z = torch.from_numpy(np.stack(zs, -1).astype(np.float32)).to(X.device)
        x = mu + std * z
        res["act"] = x
    else:
        x = actc_in
    zz = (x - mu) / std
    res["logp"] = (-0.5 * zz * zz - log_std - HALF_LOG_2PI).sum(-1)
    res["entropy"] = (0.5 + HALF_LOG_2PI + log_std).sum(-1).expand(B)
    res["mean"] = mu
    return res


def normalize_adv(adv, adv_stats):
    if adv_stats is None:
        return adv
    n = torch.clamp(adv_stats[2], min=1.0)
    mean = adv_stats[0] / n
    var = torch.clamp(adv_stats[1] / n - mean * mean, min=0.0)
    return (adv - mean) / (torch.sqrt(var) + 1e-8)


def mlp_grad_ref(head, params, X, A, H, mask=None, act=None, actc=None, adv=None, ret=None, logp_old=None,
                 adv_stats=None, inv_B=None, clip_eps=0.2, ent_coef=0.0, dtype=torch.float32):
    """Returns (flat gradient, stats dict) of sum_i loss_i * inv_B (+ entropy bonus);
    ``dtype=torch.float64`` gives the float64 oracle (tools/grad_fuzz_probe.py)."""
    B, D = X.shape
    gaussian = head in (HEAD_PPO_GAUSS, HEAD_PG_GAUSS)
    Aeff = 1 if head == HEAD_VALUE_MSE else A
    if inv_B is None:
        inv_B = 1.0 / max(B, 1)
    p = params.detach().to(dtype).clone().requires_grad_(True)
    out, log_std = trunk(p, X.to(dtype), D, H, Aeff, gaussian)
    stats = {}
    if head == HEAD_VALUE_MSE:
        v = out[:, 0]
        li = (v - ret) ** 2
        loss = li.sum() * inv_B
        stats.update(loss=li.sum().item(), v=v.sum().item(), count=B)
    else:
        advn = normalize_adv(adv.to(dtype), None if adv_stats is None else adv_stats.to(dtype))
        if not gaussian:
            logits = masked_logits(out, mask)
            logp_all = torch.log_softmax(logits, dim=-1)
            logp = logp_all.gather(-1, act.long().unsqueeze(-1)).squeeze(-1)
            pr = torch.exp(logp_all)
            ent = -(pr * torch.where(pr > 0, logp_all, torch.zeros_like(logp_all))).sum(-1)
        else:
            std = torch.exp(log_std)
            zz = (actc - out) / std
            logp = (-0.5 * zz * zz - log_std - HALF_LOG_2PI).sum(-1)
            ent = (0.5 + HALF_LOG_2PI + log_std).sum(-1).expand(B)
        if head in (HEAD_PG_CAT, HEAD_PG_GAUSS):
            li = -logp * advn
        else:
            ratio = torch.exp(logp - logp_old)
            s1 = ratio * advn
            s2 = torch.clamp(ratio, 1 - clip_eps, 1 + clip_eps) * advn
            li = -torch.minimum(s1, s2)
            stats["clipfrac"] = ((ratio - 1).abs() > clip_eps).float().sum().item()
        loss = li.sum() * inv_B - ent_coef * ent.sum() * inv_B
        stats.update(loss=li.sum().item(), entropy=ent.sum().item(), count=B)
        if logp_old is not None:
            stats["kl"] = (logp_old - logp).sum().item()
    loss.backward()
    return p.grad.detach(), stats


def discount_cumsum(x: np.ndarray, discount: float) -> np.ndarray:
    """scipy-free equivalent of BaseReplayBuffer.discount_cumsum (lfilter reversed)."""
    out = np.zeros_like(x, dtype=np.float64)
    run = 0.0
    for t in range(len(x) - 1, -1, -1):
        run = x[t] + discount * run
        out[t] = run
    return out


@torch.no_grad()
def gae_scan_tm_ref(rew, done, val, gamma, lam, tval=None):
    """done codes: 0 running, 1 terminal, 2 time-limit truncation (bootstrap tval[t]).

    [K, T, N] inputs (K actor blocks) with flat ``val`` [K*T*N + K*N] are scanned as one
    [T, K*N] problem (column k*N + n)."""
    if rew.dim() == 3:
        K, T, N = rew.shape
        tm = lambda x: x.reshape(K, T, N).permute(1, 0, 2).reshape(T, K * N)  # noqa: E731
        v = None
        if val is not None:
            vf = val.reshape(-1)
            v = torch.cat([tm(vf[:K * T * N]), vf[K * T * N:K * T * N + K * N].reshape(1, K * N)])
        a, r, s = gae_scan_tm_ref(tm(rew), tm(done), v, gamma, lam, None if tval is None else tm(tval))
        back = lambda x: x.reshape(T, K, N).permute(1, 0, 2).contiguous()  # noqa: E731
        return back(a), back(r), s
    T, N = rew.shape
    if val is not None:
        val = val.reshape(T + 1, N)
    adv = torch.zeros_like(rew)
    ret = torch.zeros_like(rew)
    if val is not None:
        v_next = val[T].clone()
        adv_next = torch.zeros(N, dtype=rew.dtype, device=rew.device)
        ret_next = v_next.clone()
        for t in range(T - 1, -1, -1):
            nd = (done[t] == 0).to(rew.dtype)
            vb = torch.where(done[t] > 1.5, tval[t], torch.zeros_like(rew[t])) if tval is not None \
                else torch.zeros_like(rew[t])
            delta = rew[t] + gamma * (v_next * nd + vb) - val[t]
            adv[t] = delta + gamma * lam * nd * adv_next
            ret[t] = rew[t] + gamma * (nd * ret_next + vb)
            adv_next, ret_next, v_next = adv[t], ret[t], val[t]
    else:
        adv_next = torch.zeros(N, dtype=rew.dtype, device=rew.device)
        ret_next = torch.zeros(N, dtype=rew.dtype, device=rew.device)
        for t in range(T - 1, -1, -1):
            nd = (done[t] == 0).to(rew.dtype)
            adv[t] = rew[t] + gamma * lam * nd * adv_next
            ret[t] = rew[t] + gamma * nd * ret_next
            adv_next, ret_next = adv[t], ret[t]
    stats = torch.stack([adv.sum(), (adv * adv).sum(), torch.tensor(float(T * N), device=rew.device)])
    return adv, ret, stats


@torch.no_grad()
def scan_flat_ref(rew, done, val, boot, gamma, lam):
    """Per-path finish_path semantics over a flat buffer (replay_buffer.py:48-79)."""
    r = rew.detach().cpu().double().numpy()
    d = done.detach().cpu().numpy() > 0
    v = None if val is None else val.detach().cpu().double().numpy()
    b = None if boot is None else boot.detach().cpu().double().numpy()
    L = len(r)
    adv = np.zeros(L)
    ret = np.zeros(L)
    start = 0
    for t in range(L):
        if d[t] or t == L - 1:
            sl = slice(start, t + 1)
            last = float(b[t]) if (b is not None and d[t]) else 0.0
            if v is not None:
                rr = np.append(r[sl], last)
                vv = np.append(v[sl], last)
                deltas = rr[:-1] + gamma * vv[1:] - vv[:-1]
                adv[sl] = discount_cumsum(deltas, gamma * lam)
                ret[sl] = discount_cumsum(rr, gamma)[:-1]
            else:
                adv[sl] = discount_cumsum(r[sl], gamma * lam)
                ret[sl] = discount_cumsum(r[sl], gamma)
            start = t + 1
    a = torch.from_numpy(adv.astype(np.float32)).to(rew.device)
    rt = torch.from_numpy(ret.astype(np.float32)).to(rew.device)
    stats = torch.tensor([adv.sum(), (adv * adv).sum(), float(L)], dtype=torch.float32, device=rew.device)
    return a, rt, stats


@torch.no_grad()
def adam_ref(param, m, v, grad, step, lr, beta1=0.9, beta2=0.999, eps=1e-8, weight_decay=0.0):
    """In-place torch.optim.Adam math on flat tensors; `step` is the new step count."""
    g = grad
    if weight_decay:
        g = g + weight_decay * param
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    bc1 = 1 - beta1**step
    bc2 = 1 - beta2**step
    denom = (v.sqrt() / (bc2**0.5)).add_(eps)
    param.addcdiv_(m, denom, value=-lr / bc1)
