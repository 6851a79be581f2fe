"""On-device vectorised actor + learner (the flagship training step).

One epoch on each rank (one process per GPU):

  1. fused rollout kernel: T steps x N envs of policy forward + Philox sampling + env
     physics, written time-major into HBM            (csrc/kernels/rollout.hip)
  2. value forward over the (T+1) x N observations    (mlp_forward VALUE)   [baseline]
  3. GAE / discounted-return scan + adv statistics    (scan.hip)
  4. all-reduce of the 3-float advantage statistics   (RCCL)                 [world > 1]
  5. fused policy fwd+bwd -> slab -> (all-reduce) -> fused Adam              (1 step)
  6. train_vf_iters x fused value fwd+bwd -> Adam, captured as one hipGraph  [baseline]

This is REINFORCE.receive_trajectory + train_model (REINFORCE.py:70-125) restated for a
GPU: the "traj_per_epoch" complete trajectories of the reference become N x T
transitions from N envs, and the per-episode finish_path becomes one scan over the
time-major buffer with done flags.  Data-parallel scaling: every rank runs its own
envs; gradients are summed with one all-reduce per optimiser step (global mean).
"""
from __future__ import annotations

import math
import time
from dataclasses import asdict, dataclass, field
from typing import Optional

import torch

from ..algorithms.core import FlatNet, ValueLoop
from ..ops import FwdMode, GradHead, MLPSpec, gae_scan_tm, grad_slabs, hip, mlp_forward, mlp_grad
from ..parallel.comm import Comm

DEVICE_ENVS = {"CartPole-v1": 0, "MountainCar-v0": 1, "Acrobot-v1": 2}


@dataclass
class VecTrainerConfig:
    env: str = "CartPole-v1"
    num_envs: int = 32768          # envs per rank
    rollout_len: int = 64          # T
    hidden: int = 128              # reference: [128, 128] (REINFORCE.py:46,49)
    with_baseline: bool = True
    gamma: float = 0.98            # reference defaults (default_config.json:3-16)
    lam: float = 0.97
    pi_lr: float = 3e-4
    vf_lr: float = 1e-3
    train_vf_iters: int = 80
    seed: int = 1
    use_graphs: bool = True
    ent_coef: float = 0.0
    max_episode_steps: Optional[int] = None

    def to_dict(self):
        return asdict(self)


class VecTrainer:
    def __init__(self, cfg: VecTrainerConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        assert self.device.type == "cuda", "the vectorised trainer runs the fused HIP rollout kernel"
        if cfg.env not in DEVICE_ENVS:
            raise ValueError(f"no device implementation of env {cfg.env!r}; have {list(DEVICE_ENVS)}")
        self.env_id = DEVICE_ENVS[cfg.env]
        h = hip()
        D, A, NS, max_steps = h.env_dims(self.env_id)
        self.D, self.A, self.NS = D, A, NS
        self.max_steps = cfg.max_episode_steps or max_steps
        N, T, H = cfg.num_envs, cfg.rollout_len, cfg.hidden
        dev = self.device
        rank = self.comm.rank
        # identical initial weights on every rank (seeded), per-rank env RNG streams
        g = torch.Generator().manual_seed(cfg.seed)
        self.pi = FlatNet(MLPSpec(D, H, A), cfg.pi_lr, dev, g)
        self.vf = FlatNet(MLPSpec(D, H, 1), cfg.vf_lr, dev, g) if cfg.with_baseline else None
        self.env_seed = (cfg.seed * 0x9E3779B97F4A7C15 + rank * 0x632BE59BD9B4E019) & 0x7FFFFFFFFFFFFFFF
        # time-major SoA rollout buffers (HBM resident)
        self.obs = torch.zeros(T + 1, N, D, device=dev)
        self.act = torch.zeros(T, N, dtype=torch.int32, device=dev)
        self.logp = torch.zeros(T, N, device=dev)
        self.rew = torch.zeros(T, N, device=dev)
        self.done = torch.zeros(T, N, device=dev)
        self.val = torch.zeros(T + 1, N, device=dev) if cfg.with_baseline else None
        self.adv = torch.zeros(T, N, device=dev)
        self.ret = torch.zeros(T, N, device=dev)
        self.state = torch.zeros(N, NS, device=dev)
        self.ep_len = torch.zeros(N, dtype=torch.int32, device=dev)
        self.ep_ret = torch.zeros(N, device=dev)
        self.ep_stats = torch.zeros(h.rollout_grid(N), 8, device=dev)
        self.stats_part = torch.zeros(h.scan_tm_parts(N), 3, device=dev)
        self.adv_stats = torch.zeros(3, device=dev)
        B = T * N
        self.B = B
        self.global_B = B * self.comm.world
        ns = grad_slabs(B, dev)
        self.pi_slab = torch.zeros(ns, self.pi.P, device=dev)
        self.pi_loss = torch.zeros(ns, 8, device=dev)
        self.vloop = ValueLoop(self.vf, self.comm, use_graph=cfg.use_graphs) if self.vf else None
        self.epoch = 0
        self.env_steps = 0  # per rank
        self._first = True

    # ------------------------------------------------------------------ one epoch
    def train_epoch(self):
        cfg, h = self.cfg, hip()
        N, T, H, A, D = cfg.num_envs, cfg.rollout_len, cfg.hidden, self.A, self.D
        step0 = self.epoch * T
        h.rollout(self.env_id, self.pi.params, H, self.state, self.ep_len, self.ep_ret, self.obs, self.act, self.logp,
                  self.rew, self.done, self.ep_stats, self.env_seed, step0, self._first, self.max_steps)
        self._first = False
        obs_all = self.obs.view((T + 1) * N, D)
        obs_b = obs_all[: T * N]
        if self.vf is not None:
            mlp_forward(FwdMode.VALUE, self.vf.params, obs_all, 1, H, out={"v": self.val.view(-1)})
        gae_scan_tm(self.rew, self.done, self.val, cfg.gamma, cfg.lam, adv=self.adv, ret=self.ret,
                    stats_part=self.stats_part, stats_out=self.adv_stats)
        self.comm.all_reduce_sum_(self.adv_stats)
        inv_B = 1.0 / self.global_B
        mlp_grad(GradHead.PG_CAT, self.pi.params, obs_b, A, H, act=self.act.view(-1), adv=self.adv.view(-1),
                 logp_old=self.logp.view(-1), adv_stats=self.adv_stats, inv_B=inv_B, ent_coef=cfg.ent_coef,
                 grad_slab=self.pi_slab, loss_slab=self.pi_loss)
        self.pi.apply(self.pi_slab, self.comm)
        if self.vf is not None:
            self.vloop.run(obs_b, self.ret.view(-1), cfg.train_vf_iters, inv_B)
        self.epoch += 1
        self.env_steps += N * T

    # ------------------------------------------------------------------ metrics
    def metrics(self) -> dict:
        """Synchronising read of the last epoch's statistics (global over ranks)."""
        ep = self.ep_stats.sum(0)
        mx = self.ep_stats[:, 3].max().reshape(1)
        mn = self.ep_stats[:, 4].min().reshape(1)
        pl = self.pi_loss.sum(0)
        vec = torch.cat([ep[:3], ep[5:6], pl[:6]])
        if self.vloop is not None:
            vf = self.vloop.loss_last.sum(0)
            v0 = self.vloop.loss_first.sum(0)
            vec = torch.cat([vec, vf[[0, 4, 5]], v0[[0]]])
        self.comm.all_reduce_sum_(vec)
        self.comm.all_reduce_max_(mx)
        self.comm.all_reduce_min_(mn)
        v = vec.tolist()
        n = max(v[0], 1.0)
        mean = v[1] / n
        out = {
            "Epoch": self.epoch,
            "AverageEpRet": mean if v[0] > 0 else float("nan"),
            "StdEpRet": math.sqrt(max(v[2] / n - mean * mean, 0.0)) if v[0] > 0 else float("nan"),
            "MaxEpRet": mx.item() if v[0] > 0 else float("nan"),
            "MinEpRet": mn.item() if v[0] > 0 else float("nan"),
            "EpLen": v[3] / n if v[0] > 0 else float("nan"),
            "Episodes": int(v[0]),
        }
        cnt = max(v[9], 1.0)
        out["LossPi"] = v[4] / cnt
        out["DeltaLossPi"] = 0.0  # both evaluated at pre-update params, as in REINFORCE.py:100-118
        out["Entropy"] = v[5] / cnt
        out["KL"] = v[6] / cnt
        if self.vloop is not None:
            vc = max(v[12], 1.0)
            out["LossV"] = v[10] / vc
            out["VVals"] = v[11] / vc
            out["DeltaLossV"] = (v[10] - v[13]) / vc
        out["EnvSteps"] = self.env_steps * self.comm.world
        out["WorldSize"] = self.comm.world
        return out

    def state_dict(self) -> dict:
        sd = {"pi": self.pi.state_dict(), "epoch": self.epoch, "env_steps": self.env_steps,
              "env_state": self.state.cpu(), "ep_len": self.ep_len.cpu(), "ep_ret": self.ep_ret.cpu(),
              "cfg": self.cfg.to_dict()}
        if self.vf is not None:
            sd["vf"] = self.vf.state_dict()
        return sd

    def load_state_dict(self, sd: dict):
        self.pi.load_state_dict(sd["pi"])
        if self.vf is not None and "vf" in sd:
            self.vf.load_state_dict(sd["vf"])
        self.epoch = int(sd["epoch"])
        self.env_steps = int(sd["env_steps"])
        self.state.copy_(sd["env_state"].to(self.device))
        self.ep_len.copy_(sd["ep_len"].to(self.device))
        self.ep_ret.copy_(sd["ep_ret"].to(self.device))
        self._first = False
