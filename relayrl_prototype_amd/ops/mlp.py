"""Flat-parameter MLP spec and device/oracle dispatch for every learner/actor op.

All networks are stored as ONE flat fp32 vector per net (``MLPSpec.P`` floats, same
order as ``nn.Sequential(Linear, ReLU, Linear, ReLU, Linear).parameters()``), so the
optimiser is a single fused launch, weight broadcast is a single collective, and the
kernels stage the whole net into LDS with one sweep.
"""
from __future__ import annotations

from dataclasses import dataclass
from enum import IntEnum
from typing import Optional

import torch

from . import reference as ref


class FwdMode(IntEnum):
    VALUE = 0
    CAT_SAMPLE = 1
    CAT_EVAL = 2
    LOGITS = 3
    GAUSS_SAMPLE = 4
    GAUSS_EVAL = 5


class GradHead(IntEnum):
    PG_CAT = 0
    VALUE_MSE = 1
    PPO_CAT = 2
    PPO_GAUSS = 3
    PG_GAUSS = 4


from ..models.mlp_spec import MLPSpec  # noqa: E402,F401 -- torch-free (CPU agents import it)


def _hip_for(t):
    from . import use_hip, hip

    return hip() if use_hip(t) else None


def _f32(t):
    return None if t is None else t.contiguous().float()


def _i32(t):
    return None if t is None else t.contiguous().to(torch.int32)


def mlp_forward(mode: int, params: torch.Tensor, X: torch.Tensor, A: int, H: int, mask=None, act_in=None,
                actc_in=None, seed: int = 0, step: int = 0, row_offset: int = 0, out: Optional[dict] = None,
                gate=None):
    """Batched fused forward.  Returns a dict with keys among v / act / logp / entropy / logits / mean.

    ``gate`` (VALUE mode): [B] done codes; the kernel evaluates only the 16-row tiles that
    contain a time-limit truncation (code 2) -- the bootstrap values of cut episodes."""
    X = X.contiguous().float()
    B = X.shape[0]
    h = _hip_for(X)
    if h is None:
        r = ref.mlp_forward_ref(int(mode), params, X, A, H, mask, act_in, actc_in, seed, step, row_offset)
        if out is not None:
            for k, v in r.items():
                if k in out:
                    out[k].copy_(v)
                else:
                    out[k] = v
            return out
        return r
    dev = X.device
    out = {} if out is None else out
    mode = int(mode)
    if mode == FwdMode.VALUE:
        v = out.get("v")
        if v is None:
            v = out["v"] = torch.empty(B, device=dev)
        h.mlp_forward(mode, params, X, A, H, None, None, None, None, None, v, None, None, seed, step, row_offset,
                      _f32(gate))
        return out
    o0 = out.setdefault("logp", torch.empty(B, device=dev))
    o1 = out.setdefault("entropy", torch.empty(B, device=dev))
    act_out = actc_out = logits = None
    if mode == FwdMode.CAT_SAMPLE:
        act_out = out.setdefault("act", torch.empty(B, dtype=torch.int32, device=dev))
    elif mode == FwdMode.LOGITS:
        logits = out.setdefault("logits", torch.empty(B, A, device=dev))
    elif mode == FwdMode.GAUSS_SAMPLE:
        actc_out = out.setdefault("act", torch.empty(B, A, device=dev))
        logits = out.setdefault("mean", torch.empty(B, A, device=dev))
    elif mode == FwdMode.GAUSS_EVAL:
        logits = out.setdefault("mean", torch.empty(B, A, device=dev))
    h.mlp_forward(mode, params, X, A, H, _f32(mask), _i32(act_in), _f32(actc_in), act_out, actc_out, o0, o1,
                  logits, seed, step, row_offset, None)
    return out


# Rows per fused fwd+bwd launch.  The grad kernels index rows x features in 32 bits (the binding
# refuses B * max(D, A) >= 2^31), so a larger batch -- the 10^8-transition HBM rollout buffers of
# BASELINE config #5 -- is launched in chunks whose gradient slabs sit back to back in one slab
# array: the fused reduce + Adam sums them all, and inv_B stays 1 / (the whole batch).
GRAD_CHUNK_ROWS = 1 << 25


def grad_chunks(B: int):
    """[(lo, hi)] row ranges of the launches for a B-row batch."""
    return [(lo, min(B, lo + GRAD_CHUNK_ROWS)) for lo in range(0, max(B, 1), GRAD_CHUNK_ROWS)]


def grad_slabs(B: int, device) -> int:
    if torch.device(device).type != "cuda":
        return 1
    from . import hip

    h = hip()
    return sum(int(h.mlp_grad_slabs(hi - lo)) for lo, hi in grad_chunks(B))


def set_value_grad_mode(mode: int) -> int:
    """Select the GPU value-MSE gradient kernel: 1 = weight-stationary bf16x6 (fp32-accurate
    split-bf16 MFMA, csrc/kernels/value_grad.hip; H = 128, D <= 8), 0 = fp32 MFMA
    (mlp_grad.hip).  -1 only queries.  Returns the previous mode."""
    from . import hip

    return int(hip().set_value_grad_mode(int(mode)))


def mlp_grad(head: int, params, X, A: int, H: int, mask=None, act=None, actc=None, adv=None, ret=None,
             logp_old=None, adv_stats=None, inv_B: Optional[float] = None, clip_eps: float = 0.2,
             ent_coef: float = 0.0, grad_slab=None, loss_slab=None, nvalid=None, inv_B_dev=None):
    """Fused forward+backward.  GPU: fills grad_slab [nslab, P] and loss_slab [nslab, 8] and
    returns them; CPU: returns (grad [1, P], loss stats [1, 8]) computed with autograd.

    ``nvalid`` (int32 [1]) / ``inv_B_dev`` (fp32 [1]): the batch shape read from device memory
    -- rows >= nvalid are inert and inv_B_dev replaces inv_B -- so a captured graph can replay
    a batch whose valid row count changes (agent rows folded into a fixed capacity)."""
    X = X.contiguous().float()
    B = X.shape[0]
    if inv_B is None:
        inv_B = 1.0 / max(B, 1)
    h = _hip_for(X)
    if h is None and (nvalid is not None or inv_B_dev is not None):
        n = B if nvalid is None else int(nvalid.reshape(-1)[0])
        ib = inv_B if inv_B_dev is None else float(inv_B_dev.reshape(-1)[0])

        def cut(t):
            return None if t is None else t[:n]

        return mlp_grad(head, params, X[:n], A, H, cut(mask), cut(act), cut(actc), cut(adv), cut(ret), cut(logp_old),
                        adv_stats, ib, clip_eps, ent_coef)
    if h is None:
        g, st = ref.mlp_grad_ref(int(head), params, X, A, H, mask, act, actc, adv, ret, logp_old, adv_stats,
                                 inv_B, clip_eps, ent_coef)
        ls = torch.zeros(1, 8)
        ls[0, 0] = st.get("loss", 0.0)
        ls[0, 1] = st.get("entropy", 0.0)
        ls[0, 2] = st.get("kl", 0.0)
        ls[0, 3] = st.get("clipfrac", 0.0)
        ls[0, 4] = st.get("v", 0.0)
        ls[0, 5] = st.get("count", B)
        return g.view(1, -1), ls
    gaussian = int(head) in (GradHead.PPO_GAUSS, GradHead.PG_GAUSS)
    Aeff = 1 if int(head) == GradHead.VALUE_MSE else A
    P = MLPSpec(X.shape[1], H, Aeff, gaussian).P
    ns = grad_slabs(B, X.device)
    if grad_slab is None:
        grad_slab = torch.empty(ns, P, device=X.device)
    if loss_slab is None:
        loss_slab = torch.empty(ns, 8, device=X.device)
    mask, act, actc, adv, ret, logp_old = _f32(mask), _i32(act), _f32(actc), _f32(adv), _f32(ret), _f32(logp_old)
    off = 0
    chunks = grad_chunks(B)
    if nvalid is not None and len(chunks) > 1:
        raise ValueError("a device-side row count needs a single-launch batch (< 2^25 rows)")
    for lo, hi in chunks:
        whole = lo == 0 and hi == B

        def rows(t):
            return t if (t is None or whole) else t[lo:hi]

        n = int(h.mlp_grad_slabs(hi - lo))
        h.mlp_grad(int(head), params, rows(X), A, H, rows(mask), rows(act), rows(actc), rows(adv), rows(ret),
                   rows(logp_old), adv_stats, float(inv_B), float(clip_eps), float(ent_coef), grad_slab[off:off + n],
                   loss_slab[off:off + n], nvalid, inv_B_dev)
        off += n
    return grad_slab[:ns], loss_slab[:ns]


def reduce_slabs(slab: torch.Tensor, scale: float = 1.0, out=None):
    if out is None:
        out = torch.empty(slab.shape[1], device=slab.device)
    h = _hip_for(slab)
    if h is None:
        out.copy_(slab.sum(0) * scale)
        return out
    h.reduce_slabs(slab.contiguous(), float(scale), out)
    return out


def adam_step(param, m, v, step_t, ticket_t, lr, grad=None, slab=None, beta1=0.9, beta2=0.999, eps=1e-8,
              grad_scale=1.0, weight_decay=0.0, grad_out=None, step_add=0, step_inc=1):
    """One fused Adam update of a flat parameter vector; `step_t` is a 1-elem int32 tensor
    holding the number of completed steps (advanced on the device).  The update uses step
    t = step_t + step_add + 1 and leaves step_t + step_inc behind: a loop of K updates passes
    (k, 0) for k < K - 1 and (K - 1, K) last, so only its last update pays the device-wide
    arrival ticket that advances the counter (adam.hip)."""
    h = _hip_for(param)
    if h is None:
        g = grad if grad is not None else slab.sum(0)
        g = g * grad_scale
        if grad_out is not None:
            grad_out.copy_(g)
        s0 = int(step_t.item())
        ref.adam_ref(param, m, v, g, s0 + step_add + 1, lr, beta1, beta2, eps, weight_decay)
        step_t.fill_(s0 + step_inc)
        return
    h.adam(param, m, v, grad, slab, grad_out, step_t, ticket_t, float(lr), float(beta1), float(beta2), float(eps),
           float(grad_scale), float(weight_decay), int(step_add), int(step_inc))


def gae_scan_tm(rew, done, val, gamma, lam, adv=None, ret=None, stats_part=None, stats_out=None, tval=None,
                stats=True, counters=()):
    """Time-major GAE / discounted-return scan -> (adv, ret, stats[3]).  ``stats=False``: the
    caller does not use the advantage statistics; the GPU path skips their reduction launch and
    returns None for them.  ``counters``: (int64 device scalar, increment) pairs (at most 3)
    advanced by the same launch (the Pong update's step counters: one launch fewer).

    ``rew`` / ``done`` / ``tval`` are [T, N], or [K, T, N] for a learner shard holding K
    actor blocks; ``val`` is flat [K*T*N + K*N]: V of every step, then the bootstrap value
    V(s_T) of each of the K*N columns (for K = 1 exactly a [T+1, N] buffer).
    done codes: 0 running, 1 terminal, 2 time-limit truncation -- bootstrapped with
    ``tval`` = V(pre-reset observation) (replay_buffer.py:48-79 last_val)."""
    h = _hip_for(rew)
    if h is None:
        a, r, s = ref.gae_scan_tm_ref(rew, done, val, gamma, lam, tval)
        if stats_out is not None:
            stats_out.copy_(s)
        for c, inc in counters:
            c += int(inc)
        return a, r, s
    K = rew.shape[0] if rew.dim() == 3 else 1
    T, N = rew.shape[-2], rew.shape[-1]
    dev = rew.device
    adv = torch.empty(rew.shape, device=dev) if adv is None else adv
    ret = torch.empty(rew.shape, device=dev) if ret is None else ret
    if stats_part is None:
        stats_part = torch.empty(int(h.scan_tm_parts(K * N)), 3, device=dev)
    if stats_out is None and stats:
        stats_out = torch.empty(3, device=dev)
    h.gae_scan_tm(rew.contiguous(), done.contiguous(), None if val is None else val.contiguous(), _f32(tval), adv, ret,
                  stats_part, stats_out, float(gamma), float(lam), counters=[(c, int(i)) for c, i in counters])
    return adv, ret, stats_out


def scan_flat(rew, done, val, boot, gamma, lam):
    """Flat concatenated-paths scan (finish_path semantics) -> (adv, ret, stats[3])."""
    h = _hip_for(rew)
    if h is None:
        return ref.scan_flat_ref(rew, done, val, boot, gamma, lam)
    L = rew.numel()
    dev = rew.device
    adv = torch.empty(L, device=dev)
    ret = torch.empty(L, device=dev)
    work = torch.empty(max(1, int(h.scan_flat_blocks(L))) * 9, device=dev)
    stats = torch.empty(3, device=dev)
    h.scan_flat(rew.contiguous().float(), done.contiguous().float(), _f32(val), _f32(boot), adv, ret, work, stats,
                float(gamma), float(lam))
    return adv, ret, stats
