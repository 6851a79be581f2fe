"""PPO-clip (the reference whitelists "PPO" in config_loader.rs:398-399 but ships no
implementation).  Clipped surrogate + approximate-KL early stopping, GAE-lambda, separate
value net; the categorical and diagonal-Gaussian heads are fused HIP kernels
(mlp_grad.hip HEAD_PPO_CAT / HEAD_PPO_GAUSS)."""
from __future__ import annotations

from .trajectory_algo import TrajectoryAlgorithm


class PPO(TrajectoryAlgorithm):
    ALGO = "ppo"
    CONFIG_NAME = "PPO"
    EXTRA_KEYS = ("hidden", "with_vf_baseline", "num_minibatches")

    def exp_name(self) -> str:
        return "relayrl-ppo-info"


class A2C(TrajectoryAlgorithm):
    """Synchronous advantage actor-critic: one policy step with an entropy bonus and
    ``train_vf_iters`` value steps per batch."""

    ALGO = "a2c"
    CONFIG_NAME = "A2C"
    EXTRA_KEYS = ("hidden", "with_vf_baseline")

    def exp_name(self) -> str:
        return "relayrl-a2c-info"
