"""Flat-parameter MLP layout (``MLPSpec``), importable without torch: CPU agents (api/agent.py,
models/cpu_policy.py) split the learner's flat weight vector with it; the device learner and
the kernels use the same offsets (ops/mlp.py re-exports it)."""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional


@dataclass(frozen=True)
class MLPSpec:
    """Linear(D,H)-ReLU-Linear(H,H)-ReLU-Linear(H,A) [+ log_std(A)]."""

    D: int
    H: int
    A: int
    gaussian: bool = False

    @property
    def P(self) -> int:
        D, H, A = self.D, self.H, self.A
        return H * D + H + H * H + H + A * H + A + (A if self.gaussian else 0)

    def offsets(self):
        D, H, A = self.D, self.H, self.A
        o = {}
        o["w1"] = 0
        o["b1"] = H * D
        o["w2"] = o["b1"] + H
        o["b2"] = o["w2"] + H * H
        o["w3"] = o["b2"] + H
        o["b3"] = o["w3"] + A * H
        o["log_std"] = o["b3"] + A
        return o

    def init(self, generator=None, device="cpu", log_std_init: float = -0.5, out_gain: Optional[float] = None):
        """nn.Linear default init (kaiming_uniform(a=sqrt(5)) == U(+-1/sqrt(fan_in)))."""
        import torch

        D, H, A = self.D, self.H, self.A
        parts = []
        for fan_in, fan_out in ((D, H), (H, H), (H, A)):
            bound = 1.0 / math.sqrt(fan_in)
            w = (torch.rand(fan_out * fan_in, generator=generator) * 2 - 1) * bound
            b = (torch.rand(fan_out, generator=generator) * 2 - 1) * bound
            if out_gain is not None and fan_out == A:
                w = w * out_gain
                b = b * 0
            parts += [w, b]
        if self.gaussian:
            parts.append(torch.full((A,), float(log_std_init)))
        return torch.cat(parts).float().to(device)

    def unflatten(self, params):
        from ..ops import reference as ref

        return ref.unflatten(params, self.D, self.H, self.A, self.gaussian)
