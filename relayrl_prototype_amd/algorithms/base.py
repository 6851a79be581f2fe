"""Plugin ABCs kept from the reference so custom algorithms port unchanged.

* AlgorithmAbstract            (_common/_algorithms/BaseAlgorithm.py:4-39)
* ForwardKernelAbstract, StepKernelAbstract, StepAndForwardKernelAbstract
                               (_common/_algorithms/BaseKernel.py:42-94)
* ReplayBufferAbstract, combined_shape, discount_cumsum, statistics_scalar
                               (_common/_algorithms/BaseReplayBuffer.py:6-82)
* ApplicationAbstract          (_common/_examples/BaseApplication.py:1-31)

Custom algorithm contract (rf/README.md:156-283, python_algorithm_reply.py:41-46):
module ``<algorithm_dir>/<NAME>/<NAME>.py`` defining class ``<NAME>`` (an
AlgorithmAbstract) whose ``save()`` writes a TorchScript model with
``step``/``get_input_dim``/``get_output_dim``.  Plugins now run in-process (no JSON
stdin/stdout bridge) and may use the HIP ops in ``relayrl_prototype_amd.ops``.
"""
from __future__ import annotations

from abc import ABC, abstractmethod

import numpy as np
import torch.nn as nn

from ..utils.logger import statistics_scalar  # noqa: F401  (re-export)


class AlgorithmAbstract(ABC):
    @abstractmethod
    def save(self) -> None:
        """Persist the current model (TorchScript) for agents."""

    @abstractmethod
    def receive_trajectory(self, trajectory) -> bool:
        """Ingest one trajectory; return True when the model was updated."""

    @abstractmethod
    def train_model(self) -> None:
        """Run one training epoch on the buffered data."""

    @abstractmethod
    def log_epoch(self) -> None:
        """Write the epoch's statistics."""


def infer_next_obs(act, obs, mask=None):
    """BaseKernel.py:6-22's placeholder model of the next observation: obs + act."""
    import torch

    return obs + torch.as_tensor(act, dtype=torch.float32)


def mlp(sizes, activation, output_activation=nn.Identity) -> nn.Sequential:
    """Linear layers of ``sizes`` with ``activation`` between them and ``output_activation``
    after the last (BaseKernel.py:25-39 contract)."""
    layers = []
    for j in range(len(sizes) - 1):
        layers.append(nn.Linear(sizes[j], sizes[j + 1]))
        layers.append((activation if j < len(sizes) - 2 else output_activation)())
    return nn.Sequential(*layers)


class ForwardKernelAbstract(nn.Module, ABC):
    @abstractmethod
    def forward(self, obs, mask, *args, **kwargs):
        ...


class StepKernelAbstract(nn.Module, ABC):
    @abstractmethod
    def step(self, obs, mask):
        ...


class StepAndForwardKernelAbstract(nn.Module, ABC):
    @abstractmethod
    def forward(self, obs, mask, *args, **kwargs):
        ...

    @abstractmethod
    def step(self, obs, mask):
        ...


class ReplayBufferAbstract(ABC):
    @abstractmethod
    def store(self, *args, **kwargs):
        ...

    @abstractmethod
    def get(self):
        ...


class ApplicationAbstract(ABC):
    @abstractmethod
    def run_application(self, *args, **kwargs):
        ...

    @abstractmethod
    def build_observation(self, *args, **kwargs):
        ...

    @abstractmethod
    def calculate_performance_return(self, *args, **kwargs):
        ...


def combined_shape(length, shape=None):
    if shape is None:
        return (length,)
    return (length, shape) if np.isscalar(shape) else (length, *shape)


def discount_cumsum(x, discount: float) -> np.ndarray:
    """y_t = sum_k discount^k x_{t+k} (scipy lfilter form, BaseReplayBuffer.py:12-27)."""
    x = np.asarray(x, dtype=np.float64)
    out = np.empty_like(x)
    run = 0.0
    for t in range(len(x) - 1, -1, -1):
        run = x[t] + discount * run
        out[t] = run
    return out
