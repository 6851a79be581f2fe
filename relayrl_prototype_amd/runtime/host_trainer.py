"""Host-env vectorised trainer: C++ env thread pool on the CPU, policy + learner on the GPU.

Per env step (north star "host-side env stepping feeds the learner
through pinned hipMemcpyAsync overlapped ..."):

   env threads write obs_t into PINNED host memory
   -> H2D copy on a side stream (non_blocking) -> fused sampling kernel (HIP)
   -> D2H actions into pinned memory -> env threads step ...

The envs are split into two halves that run in a software pipeline: while the GPU
samples actions for half B, the CPU threads step half A, so neither side idles.  The
rollout (obs, actions, log-probs) never leaves HBM for the learner; only rewards /
done flags go host -> device once per rollout.

On a CPU-only machine the same loop runs with the PyTorch oracle ops (used by the
multi-process gloo tests).
"""
from __future__ import annotations

import time
from dataclasses import asdict, dataclass
from typing import Optional

import numpy as np
import torch

from .. import _native
from ..algorithms.learner import PGLearner
from ..ops import FwdMode, mlp_forward
from ..parallel.comm import Comm
from ..utils.tracing import PhaseTimer
from .rollout_learn import RolloutLearner, episode_metrics


@dataclass
class HostTrainerConfig:
    env: str = "CartPole-v1"
    num_envs: int = 1024           # per rank (split into 2 pipeline halves)
    rollout_len: int = 128
    algo: str = "reinforce"        # reinforce | a2c | ppo
    hidden: int = 128
    with_baseline: bool = True
    gamma: float = 0.99
    lam: float = 0.95
    pi_lr: float = 3e-4
    vf_lr: float = 1e-3
    train_vf_iters: int = 80
    train_pi_iters: int = 10
    clip_ratio: float = 0.2
    target_kl: Optional[float] = None
    ent_coef: float = 0.0
    seed: int = 0
    num_threads: int = 4
    pipeline: bool = True
    use_graphs: bool = True
    log_std_init: float = -0.5
    phase_timing: bool = False

    def to_dict(self):
        return asdict(self)


class HostVecTrainer:
    def __init__(self, cfg: HostTrainerConfig, comm: Optional[Comm] = None, device=None):
        self.cfg = cfg
        self.comm = comm or Comm()
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        cuda = self.device.type == "cuda"
        N, T = cfg.num_envs, cfg.rollout_len
        halves = 2 if (cfg.pipeline and N >= 2) else 1
        self.halves = halves
        bounds = [0, N // 2, N] if halves == 2 else [0, N]
        self.bounds = bounds
        rank = self.comm.rank
        self.envs = [_native.VecEnv(cfg.env, bounds[h + 1] - bounds[h], cfg.seed * 1000003 + rank * 7919 + h,
                                    max(1, cfg.num_threads // halves)) for h in range(halves)]
        e0 = self.envs[0]
        self.D, self.A, self.continuous = e0.obs_dim, e0.act_dim, e0.continuous
        self.learner = PGLearner(cfg.algo, self.D, self.A, cfg.hidden, not self.continuous, cfg.with_baseline,
                                 cfg.pi_lr, cfg.vf_lr, cfg.train_vf_iters, cfg.train_pi_iters, cfg.clip_ratio,
                                 cfg.target_kl, cfg.ent_coef, self.device, cfg.seed, self.comm, cfg.use_graphs,
                                 cfg.log_std_init)
        self.timer = PhaseTimer(self.device, enabled=cfg.phase_timing)
        self.rl = RolloutLearner(self.learner, T, N, cfg.gamma, cfg.lam, self.comm, self.timer)
        pin = cuda
        D, A = self.D, self.A
        # pinned host staging (env side) and HBM rollout buffers (learner side)
        self.h_obs = torch.zeros(T + 1, N, D, pin_memory=pin)
        self.h_rew = torch.zeros(T, N, pin_memory=pin)
        self.h_done = torch.zeros(T, N, pin_memory=pin)  # 0 / 1 terminal / 2 time-limit truncation
        # pre-reset observations of truncated steps (bootstrap V(s_T) of cut episodes)
        self.h_tobs = torch.zeros(T, N, D, pin_memory=pin) if self.learner.vf is not None else None
        self.d_tobs = torch.zeros(T, N, D, device=self.device) if self.learner.vf is not None else None
        if self.continuous:
            self.h_act = torch.zeros(T, N, A, pin_memory=pin)
            self.d_act = torch.zeros(T, N, A, device=self.device)
        else:
            self.h_act = torch.zeros(T, N, dtype=torch.int32, pin_memory=pin)
            self.d_act = torch.zeros(T, N, dtype=torch.int32, device=self.device)
        self.d_obs = torch.zeros(T + 1, N, D, device=self.device)
        self.d_logp = torch.zeros(T, N, device=self.device)
        self.d_rew = torch.zeros(T, N, device=self.device)
        self.d_done = torch.zeros(T, N, device=self.device)
        self.copy_stream = torch.cuda.Stream(self.device) if cuda else None
        # first observation
        for h, env in enumerate(self.envs):
            lo = bounds[h]
            env.reset_ptr(self.h_obs[0, lo].data_ptr())
        self.epoch = 0
        self.env_steps = 0
        self.global_step = 0
        self.timings = {"rollout_s": 0.0, "learn_s": 0.0}

    def _sample(self, t, h):
        lo, hi = self.bounds[h], self.bounds[h + 1]
        cuda = self.device.type == "cuda"
        mode = FwdMode.GAUSS_SAMPLE if self.continuous else FwdMode.CAT_SAMPLE
        seed = (self.cfg.seed * 0x9E3779B9 + self.comm.rank * 0x85EBCA6B) & 0x7FFFFFFFFFFF
        if cuda:
            cs = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self.copy_stream):
                self.d_obs[t, lo:hi].copy_(self.h_obs[t, lo:hi], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(self.copy_stream)
            cs.wait_event(ev)
            out = {"logp": self.d_logp[t, lo:hi]}
            if self.continuous:
                out["act"] = self.d_act[t, lo:hi]
                out["mean"] = torch.empty(hi - lo, self.A, device=self.device)
            else:
                out["act"] = self.d_act[t, lo:hi]
            mlp_forward(mode, self.learner.pi.params, self.d_obs[t, lo:hi], self.A, self.cfg.hidden, seed=seed,
                        step=self.global_step + t, row_offset=lo, out=out)
            self.h_act[t, lo:hi].copy_(self.d_act[t, lo:hi], non_blocking=True)
            done_ev = torch.cuda.Event()
            done_ev.record(cs)
            return done_ev
        self.d_obs[t, lo:hi].copy_(self.h_obs[t, lo:hi])
        r = mlp_forward(mode, self.learner.pi.params, self.d_obs[t, lo:hi], self.A, self.cfg.hidden, seed=seed,
                        step=self.global_step + t, row_offset=lo)
        self.d_act[t, lo:hi].copy_(r["act"])
        self.d_logp[t, lo:hi].copy_(r["logp"])
        self.h_act[t, lo:hi].copy_(r["act"])
        return None

    def _step_env(self, t, h):
        lo = self.bounds[h]
        self.envs[h].step_ptr(self.h_act[t, lo].data_ptr(), self.h_obs[t + 1, lo].data_ptr(),
                              self.h_rew[t, lo].data_ptr(), self.h_done[t, lo].data_ptr(),
                              self.h_tobs[t, lo].data_ptr() if self.h_tobs is not None else 0)

    def rollout(self):
        T = self.cfg.rollout_len
        t0 = time.perf_counter()
        for t in range(T):
            evs = [self._sample(t, h) for h in range(self.halves)]
            for h in range(self.halves):
                if evs[h] is not None:
                    evs[h].synchronize()  # actions of half h are on the host; half h+1 still sampling
                self._step_env(t, h)
        # last observation + rewards / dones to the device (async on the copy stream)
        if self.device.type == "cuda":
            with torch.cuda.stream(self.copy_stream):
                self.d_obs[T].copy_(self.h_obs[T], non_blocking=True)
                self.d_rew.copy_(self.h_rew, non_blocking=True)
                self.d_done.copy_(self.h_done, non_blocking=True)
                if self.d_tobs is not None:
                    self.d_tobs.copy_(self.h_tobs, non_blocking=True)
            torch.cuda.current_stream(self.device).wait_stream(self.copy_stream)
        else:
            self.d_obs[T].copy_(self.h_obs[T])
            self.d_rew.copy_(self.h_rew)
            self.d_done.copy_(self.h_done)
            if self.d_tobs is not None:
                self.d_tobs.copy_(self.h_tobs)
        self.global_step += T
        self.timings["rollout_s"] += time.perf_counter() - t0

    def train_epoch(self):
        with self.timer.phase("Rollout"):
            self.rollout()
        t0 = time.perf_counter()
        self.rl.learn(self.d_obs, self.d_act, self.d_rew, self.d_done, self.d_logp, tobs=self.d_tobs)
        # next rollout starts from the last observation
        self.h_obs[0].copy_(self.h_obs[self.cfg.rollout_len])
        self.timings["learn_s"] += time.perf_counter() - t0
        self.epoch += 1
        self.env_steps += self.cfg.num_envs * self.cfg.rollout_len

    def metrics(self) -> dict:
        tot = {"n": 0.0, "sum": 0.0, "sumsq": 0.0, "max": -1e300, "min": 1e300, "sum_len": 0.0}
        for e in self.envs:
            s = e.take_stats()
            if s["n"] > 0:
                tot["max"] = max(tot["max"], s["max"])
                tot["min"] = min(tot["min"], s["min"])
            for k in ("n", "sum", "sumsq", "sum_len"):
                tot[k] += s[k]
        out = {"Epoch": self.epoch}
        out.update(episode_metrics(self.comm, tot["n"], tot["sum"], tot["sumsq"], tot["max"], tot["min"],
                                   tot["sum_len"]))
        out.update(self.learner.summarize())
        out["EnvSteps"] = self.env_steps * self.comm.world
        out["WorldSize"] = self.comm.world
        out["RolloutS"] = self.timings["rollout_s"]
        out["LearnS"] = self.timings["learn_s"]
        if self.timer.enabled:
            out.update(self.timer.columns())
            self.timer.reset()
        return out
