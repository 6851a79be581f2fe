"""Agent-side runner for an arbitrary TorchScript policy -- the reference's model contract.

The reference agent holds a ``CModule`` and calls its exported ``step(obs, mask)`` for every
action (agent_zmq.rs:458-520, agent_grpc.rs:398): obs and mask are cast to float, ``step``
runs under ``no_grad`` and returns ``(action Tensor, Dict[str, Tensor | int | float])``.  A
model is accepted only after ``validate_model`` (agent_wrapper.rs:88-168): integer
``get_input_dim`` / ``get_output_dim`` and a dummy ``step`` on ``[1, input_dim]`` zeros that
returns a 2-tuple of a Tensor and a NON-empty dict.  The dict becomes the action's aux data
through ``convert_generic_dict`` (agent_wrapper.rs:186-211): tensors as float32, ints, floats;
other values are dropped.

This is the path for custom algorithm plugins (rf/README.md:156-229), whose networks can be
anything.  The built-in MLP layout keeps its native fast path (models/cpu_policy.py, C++),
which needs no TorchScript interpreter at all.  The README's ``get_obs_dim`` / ``get_act_dim``
names are accepted in place of ``get_input_dim`` / ``get_output_dim``.
"""
from __future__ import annotations

import io
import threading
from typing import Any, Dict, Optional, Tuple

import numpy as np


def _dim(module, names) -> int:
    for n in names:
        fn = getattr(module, n, None)
        if fn is None:
            continue
        v = fn()
        if isinstance(v, bool) or not isinstance(v, int):
            raise TypeError(f"{n}() must return an int, got {type(v).__name__}")
        if v < 0:
            raise ValueError(f"{n}() must be non-negative, got {v}")
        return int(v)
    raise AttributeError(f"model exports none of {names} (agent_wrapper.rs:88-120)")


def convert_generic_dict(d) -> Dict[str, Any]:
    """agent_wrapper.rs:186-211: str keys; Tensor -> float32 ndarray, int, float; others dropped."""
    import torch

    out: Dict[str, Any] = {}
    for k, v in d.items():
        if not isinstance(k, str):
            continue
        if isinstance(v, torch.Tensor):
            out[k] = v.detach().to(torch.float32).cpu().numpy()
        elif isinstance(v, bool):
            continue
        elif isinstance(v, int):
            out[k] = int(v)
        elif isinstance(v, float):
            out[k] = float(v)
    return out


def validate_model(module) -> Tuple[int, int]:
    """agent_wrapper.rs:88-168 -> (input_dim, output_dim); raises ValueError on a bad model."""
    import torch

    try:
        in_dim = _dim(module, ("get_input_dim", "get_obs_dim"))
        out_dim = _dim(module, ("get_output_dim", "get_act_dim"))
        with torch.no_grad():
            res = module.step(torch.zeros(1, in_dim, dtype=torch.float32), torch.zeros(1, out_dim, dtype=torch.float32))
    except (AttributeError, TypeError, RuntimeError) as e:
        raise ValueError(f"model validation failed: {e}") from e
    if not isinstance(res, tuple) or len(res) != 2:
        raise ValueError("model validation failed: step must return a tuple of length 2")
    if not isinstance(res[0], torch.Tensor):
        raise ValueError("model validation failed: the first element of step's tuple must be a Tensor")
    if not isinstance(res[1], dict) or not res[1]:
        raise ValueError("model validation failed: the second element of step's tuple must be a non-empty dict")
    return in_dim, out_dim


class TorchScriptPolicy:
    """The CPUPolicy interface (``step`` / ``value`` / dims / ``version``) over a TorchScript
    module.  ``step`` returns ``(act ndarray [1, ...], data dict of ndarrays / scalars)``."""

    is_torchscript = True
    hidden = -1  # no MLP layout

    def __init__(self, archive: bytes, seed: Optional[int] = None):
        import torch

        self.archive = bytes(archive)
        self.module = torch.jit.load(io.BytesIO(self.archive), map_location="cpu")
        self.module.eval()
        self.obs_dim, self.act_dim = validate_model(self.module)
        self.version = 0
        self._gen_lock = threading.Lock()
        if seed is not None:
            torch.manual_seed(int(seed))

    def step(self, obs, mask):
        import torch

        o = torch.from_numpy(np.ascontiguousarray(obs, np.float32))
        m = torch.from_numpy(np.ascontiguousarray(mask, np.float32))
        with torch.no_grad():
            act, data = self.module.step(o, m)
        a = act.detach().to(torch.float32).cpu().numpy()
        if a.ndim == 0:
            a = a.reshape(1)
        return a, convert_generic_dict(data)

    def value(self, obs) -> Optional[np.ndarray]:
        """V(obs) when the model's ``step`` reports one as ``data["v"]`` (the reference
        PolicyWithBaseline does, kernel.py:107-116); None otherwise."""
        mask = np.ones((np.asarray(obs).shape[0] if np.asarray(obs).ndim > 1 else 1, self.act_dim), np.float32)
        _, data = self.step(np.asarray(obs, np.float32).reshape(mask.shape[0], -1), mask)
        v = data.get("v")
        return None if v is None else np.asarray(v, np.float32).reshape(-1)
