"""Device ops: gfx950 HIP kernels with a pure-PyTorch fp32 oracle.

``hip()`` returns the compiled extension (``_hip_ops``).  On a machine with a GPU the
HIP path is mandatory: if the in-tree extension is missing or fails to load we raise
instead of silently falling back to PyTorch, so a GPU run can never pass on the oracle.
CPU tensors always go through :mod:`relayrl_prototype_amd.ops.reference`.
"""
from __future__ import annotations

import importlib

_HIP = None
_HIP_ERR = None


class NativeExtensionMissing(RuntimeError):
    pass


def _load():
    global _HIP, _HIP_ERR
    if _HIP is not None or _HIP_ERR is not None:
        return _HIP
    try:
        import torch  # noqa: F401  (loads libamdhip64 / libc10_hip first)

        _HIP = importlib.import_module("relayrl_prototype_amd._hip_ops")
    except Exception as e:  # pragma: no cover - depends on the build
        _HIP_ERR = e
    return _HIP


def hip():
    """The HIP extension module; raises NativeExtensionMissing if it cannot be loaded."""
    m = _load()
    if m is None:
        raise NativeExtensionMissing(
            "relayrl_prototype_amd._hip_ops is not built or failed to load "
            f"({_HIP_ERR!r}); run `python -m relayrl_prototype_amd._build`"
        )
    return m


def hip_available() -> bool:
    return _load() is not None


def use_hip(t) -> bool:
    """True when tensor ``t`` lives on the GPU (then the HIP kernel MUST be used)."""
    if not getattr(t, "is_cuda", False):
        return False
    hip()  # loud failure when missing on a GPU box
    return True


from .mlp import (  # noqa: E402
    MLPSpec,
    FwdMode,
    GradHead,
    mlp_forward,
    mlp_grad,
    set_value_grad_mode,
    grad_slabs,
    adam_step,
    reduce_slabs,
    gae_scan_tm,
    scan_flat,
)

__all__ = [
    "hip",
    "hip_available",
    "use_hip",
    "NativeExtensionMissing",
    "MLPSpec",
    "FwdMode",
    "GradHead",
    "mlp_forward",
    "mlp_grad",
    "set_value_grad_mode",
    "grad_slabs",
    "adam_step",
    "reduce_slabs",
    "gae_scan_tm",
    "scan_flat",
]
