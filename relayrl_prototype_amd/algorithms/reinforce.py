"""REINFORCE (+ optional value baseline) -- reference REINFORCE.py:16-160 on the HIP path."""
from __future__ import annotations

from .trajectory_algo import TrajectoryAlgorithm


class REINFORCE(TrajectoryAlgorithm):
    ALGO = "reinforce"
    CONFIG_NAME = "REINFORCE"

    def exp_name(self) -> str:
        # REINFORCE.py:53-57
        return "relayrl-reinforce-vf-info" if self.with_baseline else "relayrl-reinforce-info"
