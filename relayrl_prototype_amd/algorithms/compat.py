"""Import paths of the reference's plugin SDK, so reference-style plugins load unchanged.

A reference plugin (rf/README.md:200-229, algorithms/REINFORCE/REINFORCE.py:1-13) imports

    from _common._algorithms.BaseAlgorithm import AlgorithmAbstract
    from _common._algorithms.BaseKernel import mlp, StepKernelAbstract, ...
    from _common._algorithms.BaseReplayBuffer import ReplayBufferAbstract, discount_cumsum, ...
    from _common._examples.BaseApplication import ApplicationAbstract
    from utils.logger import EpochLogger, setup_logger_kwargs
    from relayrl_framework import RelayRLTrajectory, ConfigLoader

``install_reference_aliases()`` registers those module names in ``sys.modules`` as views of
this package (algorithms/base.py, utils/logger.py); ``relayrl_framework`` is a real shim
package at the repository root.  ``utils`` is aliased only when no other top-level ``utils``
is importable, so a user's own package of that name wins.
"""
from __future__ import annotations

import importlib.util
import sys
import types

_INSTALLED = False


def _module(name: str, doc: str, **attrs) -> types.ModuleType:
    m = types.ModuleType(name, doc)
    m.__dict__.update(attrs)
    return m


def install_reference_aliases() -> None:
    global _INSTALLED
    if _INSTALLED:
        return
    from . import base
    from ..utils import logger

    pkg = lambda n: _module(n, f"relayrl_prototype_amd alias of the reference's {n}", __path__=[])  # noqa: E731
    mods = {
        "_common": pkg("_common"),
        "_common._algorithms": pkg("_common._algorithms"),
        "_common._examples": pkg("_common._examples"),
        "_common._algorithms.BaseAlgorithm": _module(
            "_common._algorithms.BaseAlgorithm", base.__doc__, AlgorithmAbstract=base.AlgorithmAbstract),
        "_common._algorithms.BaseKernel": _module(
            "_common._algorithms.BaseKernel", base.__doc__, mlp=base.mlp, infer_next_obs=base.infer_next_obs,
            ForwardKernelAbstract=base.ForwardKernelAbstract, StepKernelAbstract=base.StepKernelAbstract,
            StepAndForwardKernelAbstract=base.StepAndForwardKernelAbstract),
        "_common._algorithms.BaseReplayBuffer": _module(
            "_common._algorithms.BaseReplayBuffer", base.__doc__, ReplayBufferAbstract=base.ReplayBufferAbstract,
            combined_shape=base.combined_shape, discount_cumsum=base.discount_cumsum,
            statistics_scalar=base.statistics_scalar),
        "_common._examples.BaseApplication": _module(
            "_common._examples.BaseApplication", base.__doc__, ApplicationAbstract=base.ApplicationAbstract),
    }
    for name, m in mods.items():
        sys.modules.setdefault(name, m)
    for parent, child in (("_common", "_algorithms"), ("_common", "_examples")):
        setattr(sys.modules[parent], child, sys.modules[f"{parent}.{child}"])
    for sub in ("BaseAlgorithm", "BaseKernel", "BaseReplayBuffer"):
        setattr(sys.modules["_common._algorithms"], sub, sys.modules[f"_common._algorithms.{sub}"])
    setattr(sys.modules["_common._examples"], "BaseApplication", sys.modules["_common._examples.BaseApplication"])
    if "utils" not in sys.modules and importlib.util.find_spec("utils") is None:
        u = pkg("utils")
        u.logger = logger
        sys.modules["utils"] = u
        sys.modules["utils.logger"] = logger
    _INSTALLED = True
