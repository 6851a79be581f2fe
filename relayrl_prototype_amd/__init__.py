"""relayrl_prototype_amd -- MI355X-native actor/learner RL engine.

Python API parity with jrcalgo/RelayRL-prototype (relayrl_framework/src/lib.rs:163-186):
``ConfigLoader``, ``TrainingServer``, ``RelayRLAgent``, ``RelayRLTrajectory``,
``RelayRLAction``.  The compute path is hand-written gfx950 HIP (``ops``), the runtime
is C++ (``_native``), multi-GPU uses RCCL through ``torch.distributed``.
"""
__version__ = "0.1.0"

_LAZY = {
    "ConfigLoader": ("relayrl_prototype_amd.config", "ConfigLoader"),
    "RelayRLAction": ("relayrl_prototype_amd.types", "RelayRLAction"),
    "RelayRLTrajectory": ("relayrl_prototype_amd.types", "RelayRLTrajectory"),
    "TrainingServer": ("relayrl_prototype_amd.api.server", "TrainingServer"),
    "RelayRLAgent": ("relayrl_prototype_amd.api.agent", "RelayRLAgent"),
}

__all__ = list(_LAZY)


def __getattr__(name):
    if name in _LAZY:
        import importlib

        mod, attr = _LAZY[name]
        return getattr(importlib.import_module(mod), attr)
    raise AttributeError(name)
