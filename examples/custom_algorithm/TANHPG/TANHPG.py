"""A custom algorithm written to the reference's plugin contract (rf/README.md:156-229) and
nothing else: its own network (3 x 64 tanh, NOT the built-in [128, 128] layout), its own
Python replay buffer, its own PyTorch training, and a ``save()`` that writes TorchScript.

    TrainingServer("TANHPG", obs_dim, act_dim, buf_size, algorithm_dir="examples/custom_algorithm")

The server calls ``receive_trajectory`` for every upload (reference per-action layout: actions
with ``done=False`` and their ``step()`` dicts, closed by a ``done`` marker whose reward is the
bootstrap value), and after each update that returns True it calls ``save()`` and ships the
file's bytes to every agent, which runs this module's ``step`` (models/ts_policy.py).
"""
import numpy as np
import torch
import torch.nn as nn
from torch.optim import Adam

from _common._algorithms.BaseAlgorithm import AlgorithmAbstract
from _common._algorithms.BaseKernel import StepKernelAbstract, mlp
from _common._algorithms.BaseReplayBuffer import ReplayBufferAbstract, discount_cumsum
from relayrl_framework import ConfigLoader, RelayRLTrajectory
from utils.logger import EpochLogger, setup_logger_kwargs


class TanhPolicy(StepKernelAbstract):
    def __init__(self, obs_dim: int, act_dim: int, hidden: int = 64):
        super().__init__()
        self.input_dim = obs_dim
        self.output_dim = act_dim
        self.pi = mlp([obs_dim, hidden, hidden, hidden, act_dim], nn.Tanh)
        self.v = mlp([obs_dim, hidden, hidden, hidden, 1], nn.Tanh)

    def forward(self, obs: torch.Tensor, mask: torch.Tensor):
        return self.pi(obs) + (mask - 1.0) * 1e8

    @torch.jit.export
    def step(self, obs: torch.Tensor, mask: torch.Tensor):
        with torch.no_grad():
            logits = self.forward(obs, mask)
            logp_all = torch.log_softmax(logits, dim=-1)
            act = torch.multinomial(logp_all.exp(), 1)
            logp_a = logp_all.gather(-1, act).squeeze(-1)
            v = self.v(obs).squeeze(-1)
        data = {"logp_a": logp_a, "v": v}
        return act.squeeze(-1).to(torch.float32), data

    @torch.jit.export
    def get_obs_dim(self) -> int:
        return self.input_dim

    @torch.jit.export
    def get_act_dim(self) -> int:
        return self.output_dim


class EpisodeBuffer(ReplayBufferAbstract):
    def __init__(self, gamma: float):
        self.gamma = gamma
        self.obs, self.act, self.mask, self.ret, self.adv = [], [], [], [], []
        self._rew, self._val = [], []

    def store(self, obs, act, mask, rew, val):
        self.obs.append(np.asarray(obs, np.float32).reshape(-1))
        self.act.append(int(np.asarray(act).reshape(-1)[0]))
        self.mask.append(np.asarray(mask, np.float32).reshape(-1))
        self._rew.append(float(rew))
        self._val.append(float(val))

    def finish_path(self, last_val: float = 0.0):
        rews = np.append(np.asarray(self._rew, np.float32), last_val)
        ret = discount_cumsum(rews, self.gamma)[:-1]
        self.ret.extend(ret.tolist())
        self.adv.extend((ret - np.asarray(self._val)).tolist())
        self._rew, self._val = [], []

    def get(self):
        adv = np.asarray(self.adv, np.float32)
        adv = (adv - adv.mean()) / (adv.std() + 1e-8)
        out = {"obs": torch.as_tensor(np.stack(self.obs)), "act": torch.as_tensor(self.act),
               "mask": torch.as_tensor(np.stack(self.mask)), "ret": torch.as_tensor(self.ret, dtype=torch.float32),
               "adv": torch.as_tensor(adv)}
        self.obs, self.act, self.mask, self.ret, self.adv = [], [], [], [], []
        return out


class TANHPG(AlgorithmAbstract):
    def __init__(self, env_dir: str, config_path: str, obs_dim: int, act_dim: int, buf_size: int):
        super().__init__()
        config_loader = ConfigLoader(algorithm_name="TANHPG", config_path=config_path)
        hp = (config_loader.get_algorithm_params() or {}).get("TANHPG", {})
        self.save_model_path = config_loader.get_server_model_path()
        self.traj_per_epoch = int(hp.get("traj_per_epoch", 4))
        self.train_vf_iters = int(hp.get("train_vf_iters", 5))
        torch.manual_seed(int(hp.get("seed", 1)))
        self._model = TanhPolicy(obs_dim, act_dim)
        self._pi_opt = Adam(self._model.pi.parameters(), lr=float(hp.get("pi_lr", 1e-2)))
        self._vf_opt = Adam(self._model.v.parameters(), lr=float(hp.get("vf_lr", 1e-2)))
        self._buf = EpisodeBuffer(float(hp.get("gamma", 0.99)))
        self.logger = EpochLogger(**setup_logger_kwargs("tanhpg", seed=0, data_dir=f"{env_dir}/logs"))
        self.traj = 0
        self.epoch = 0

    def save(self) -> None:
        self._model.eval()
        torch.jit.save(torch.jit.script(self._model), self.save_model_path)
        self._model.train()

    def receive_trajectory(self, trajectory: RelayRLTrajectory) -> bool:
        self.traj += 1
        ep_ret, ep_len = 0.0, 0
        for a in trajectory.get_actions():
            if not a.get_done():
                data = a.get_data()
                self._buf.store(a.get_obs(), a.get_act(), a.get_mask(), a.get_rew(),
                                float(np.asarray(data["v"]).reshape(-1)[0]))
                ep_ret += a.get_rew()
                ep_len += 1
            else:
                self._buf.finish_path(a.get_rew())
                self.logger.store(EpRet=ep_ret, EpLen=ep_len)
                ep_ret, ep_len = 0.0, 0
        if self.traj % self.traj_per_epoch == 0:
            self.epoch += 1
            self.train_model()
            self.log_epoch()
            return True
        return False

    def train_model(self) -> None:
        d = self._buf.get()
        logits = self._model(d["obs"], d["mask"])
        logp = torch.log_softmax(logits, -1).gather(-1, d["act"].long().unsqueeze(-1)).squeeze(-1)
        loss_pi = -(logp * d["adv"]).mean()
        self._pi_opt.zero_grad()
        loss_pi.backward()
        self._pi_opt.step()
        for _ in range(self.train_vf_iters):
            loss_v = ((self._model.v(d["obs"]).squeeze(-1) - d["ret"]) ** 2).mean()
            self._vf_opt.zero_grad()
            loss_v.backward()
            self._vf_opt.step()
        self.logger.store(LossPi=loss_pi.item(), LossV=loss_v.item())

    def log_epoch(self) -> None:
        self.logger.log_tabular("Epoch", self.epoch)
        self.logger.log_tabular("EpRet", with_min_and_max=True)
        self.logger.log_tabular("EpLen", average_only=True)
        self.logger.log_tabular("LossPi", average_only=True)
        self.logger.log_tabular("LossV", average_only=True)
        self.logger.dump_tabular()
