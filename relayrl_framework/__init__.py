"""Compatibility shim: ``from relayrl_framework import ...`` as in the reference
(relayrl_framework/src/lib.rs:163-186) resolves to relayrl_prototype_amd."""
from relayrl_prototype_amd import (  # noqa: F401
    ConfigLoader,
    RelayRLAction,
    RelayRLAgent,
    RelayRLTrajectory,
    TrainingServer,
)

__all__ = ["ConfigLoader", "TrainingServer", "RelayRLAgent", "RelayRLTrajectory", "RelayRLAction"]
