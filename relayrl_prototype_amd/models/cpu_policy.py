"""Agent-side policy execution on the CPU from flat weights (no TorchScript interpreter).

The reference agent runs ``CModule.method_is("step", ...)`` at batch 1 through the
TorchScript interpreter plus ~8 safetensors encodes per step.  Off-GPU
agents here evaluate the same MLP with numpy from the flat fp32 vectors the learner
broadcasts; on-GPU actors use the fused HIP kernels instead (ops.mlp_forward).
``step`` runs in C++ (csrc/host/policy.cpp, ~5 us per call incl. the value head, vs
~55 us for the numpy path); ``logits`` / ``value`` / ``step_numpy`` stay in numpy as
the readable reference the native path is tested against.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

from .mlp_spec import MLPSpec

HALF_LOG_2PI = 0.9189385332046727


class CPUPolicy:
    def __init__(self, obs_dim: int, act_dim: int, hidden: int, discrete: bool, pi_params, vf_params=None,
                 seed: int = 0):
        self.obs_dim, self.act_dim, self.hidden, self.discrete = obs_dim, act_dim, hidden, discrete
        self.rng = np.random.default_rng(seed)
        self.version = 0
        from .. import _native

        self._nat = _native.NativePolicy(obs_dim, hidden, act_dim, discrete, int(seed) & 0x7FFFFFFFFFFFFFFF)
        self.load(pi_params, vf_params)

    @staticmethod
    def _np(x):
        if x is None:
            return None
        if hasattr(x, "detach"):
            x = x.detach().cpu().numpy()
        return np.asarray(x, dtype=np.float32)

    def load(self, pi_params, vf_params=None, version: Optional[int] = None):
        sp = MLPSpec(self.obs_dim, self.hidden, self.act_dim, not self.discrete)
        p = self._np(pi_params)
        if p.size != sp.P:
            raise ValueError(f"policy params have {p.size} floats, expected {sp.P} for {sp}")
        self.pi = self._split(p, sp)
        v = self._np(vf_params)
        if v is not None:
            sv = MLPSpec(self.obs_dim, self.hidden, 1)
            if v.size != sv.P:
                raise ValueError(f"value params have {v.size} floats, expected {sv.P}")
            self.vf = self._split(v, sv)
        else:
            self.vf = None
        self._nat.load(p, v)
        if version is not None:
            self.version = version

    @staticmethod
    def _split(p, sp: MLPSpec):
        o = sp.offsets()
        D, H, A = sp.D, sp.H, sp.A
        W1 = p[o["w1"]:o["b1"]].reshape(H, D)
        b1 = p[o["b1"]:o["w2"]]
        W2 = p[o["w2"]:o["b2"]].reshape(H, H)
        b2 = p[o["b2"]:o["w3"]]
        W3 = p[o["w3"]:o["b3"]].reshape(A, H)
        b3 = p[o["b3"]:o["b3"] + A]
        ls = p[o["log_std"]:o["log_std"] + A] if sp.gaussian else None
        return (W1.T.copy(), b1, W2.T.copy(), b2, W3.T.copy(), b3, ls)

    @staticmethod
    def _trunk(net, x):
        W1t, b1, W2t, b2, W3t, b3, _ = net
        h = np.maximum(x @ W1t + b1, 0.0)
        h = np.maximum(h @ W2t + b2, 0.0)
        return h @ W3t + b3

    def logits(self, obs, mask=None):
        x = np.asarray(obs, np.float32).reshape(-1, self.obs_dim)
        out = self._trunk(self.pi, x)
        if mask is not None:
            out = out + (np.asarray(mask, np.float32).reshape(out.shape) - 1.0) * 1e8
        return out

    def value(self, obs) -> Optional[np.ndarray]:
        if self.vf is None:
            return None
        x = np.asarray(obs, np.float32).reshape(-1, self.obs_dim)
        return self._trunk(self.vf, x)[:, 0]

    def step(self, obs, mask=None) -> Tuple[np.ndarray, Dict[str, np.ndarray]]:
        """-> (act [N] int32 or [N, A] float32, {"logp_a": [N], "v": [N]?}) -- native C++."""
        act, logp, v = self._nat.step(obs, mask)
        data = {"logp_a": logp}
        if v is not None:
            data["v"] = v
        return act, data

    def step_numpy(self, obs, mask=None) -> Tuple[np.ndarray, Dict[str, np.ndarray]]:
        """numpy reference of ``step`` (different RNG stream, same distribution)."""
        x = np.asarray(obs, np.float32).reshape(-1, self.obs_dim)
        out = self._trunk(self.pi, x)
        if self.discrete:
            if mask is not None:
                out = out + (np.asarray(mask, np.float32).reshape(out.shape) - 1.0) * 1e8
            m = out.max(-1, keepdims=True)
            z = out - m
            lse = np.log(np.exp(z).sum(-1, keepdims=True))
            logp_all = z - lse
            p = np.exp(logp_all)
            u = self.rng.random((x.shape[0], 1))
            act = np.minimum((np.cumsum(p, -1) < u).sum(-1), self.act_dim - 1)
            logp = np.take_along_axis(logp_all, act[:, None], -1)[:, 0]
        else:
            ls = self.pi[6]
            std = np.exp(ls)
            act = (out + std * self.rng.standard_normal(out.shape)).astype(np.float32)
            zz = (act - out) / std
            logp = (-0.5 * zz * zz - ls - HALF_LOG_2PI).sum(-1)
        data = {"logp_a": logp.astype(np.float32)}
        v = self.value(x)
        if v is not None:
            data["v"] = v.astype(np.float32)
        return act, data
