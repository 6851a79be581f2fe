"""Shared "rollout -> returns -> optimise" step for the vectorised trainers."""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..algorithms.learner import PGLearner
from ..ops import FwdMode, gae_scan_tm, mlp_forward
from ..parallel.comm import Comm
from ..utils.tracing import PhaseTimer


class RolloutLearner:
    """Owns the HBM-resident scan buffers and drives a PGLearner on time-major rollouts."""

    def __init__(self, learner: PGLearner, T: int, N: int, gamma: float, lam: float, comm: Optional[Comm] = None,
                 timer: Optional[PhaseTimer] = None, blocks: int = 1):
        """``blocks`` = K actor rollouts per learner shard (runtime/actor_learner.py): the
        shard's batch is K time-major [T, N] blocks back to back, then the K x N final
        observations (obs rows [K*T*N + K*N]); K = 1 is the plain [T+1, N] layout."""
        self.learner = learner
        self.timer = timer or PhaseTimer(learner.device, enabled=False)
        self.T, self.N, self.K = T, N, int(blocks)
        self.gamma, self.lam = gamma, lam
        self.comm = comm or Comm()
        dev = learner.device
        K = self.K
        shape = (T, N) if K == 1 else (K, T, N)
        self.val = torch.zeros(K * (T + 1) * N, device=dev) if learner.vf is not None else None
        self.tval = torch.zeros(shape, device=dev) if learner.vf is not None else None  # V(pre-reset obs)
        self.adv = torch.zeros(shape, device=dev)
        self.ret = torch.zeros(shape, device=dev)
        self.adv_stats = torch.zeros(3, device=dev)
        self.stats_part = None
        if dev.type == "cuda":
            from ..ops import hip

            self.stats_part = torch.zeros(hip().scan_tm_parts(K * N), 3, device=dev)

    def learn(self, obs, act, rew, done, logp, mask=None, tobs=None):
        """obs [T+1, N, D] (or flat [K*T*N + K*N, D]); act [T, N] int32 or [T, N, A];
        rew / done / logp [T, N] (or [K, T, N] with the same row order as obs).

        done codes 0 / 1 / 2 = running / terminal / time-limit truncation; ``tobs`` holds the
        pre-reset observation of truncated steps, whose value bootstraps the cut episode
        (replay_buffer.py:48-79 finish_path(last_val))."""
        T, N, K = self.T, self.N, self.K
        B = K * T * N
        lr = self.learner
        D = obs.shape[-1]
        obs_all = obs.reshape(K * (T + 1) * N, D)
        obs_b = obs_all[:B]
        tm = self.timer
        with tm.phase("ValueFwd"):
            if lr.vf is not None:
                if obs_all.is_cuda:
                    mlp_forward(FwdMode.VALUE, lr.vf.params, obs_all, 1, lr.hidden, out={"v": self.val})
                else:
                    self.val.copy_(mlp_forward(FwdMode.VALUE, lr.vf.params, obs_all, 1, lr.hidden)["v"].reshape(-1))
                if tobs is not None:
                    # only the 16-row tiles holding a truncation are evaluated (gate = done codes)
                    mlp_forward(FwdMode.VALUE, lr.vf.params, tobs.reshape(B, D), 1, lr.hidden,
                                out={"v": self.tval.view(-1)}, gate=done.reshape(-1))
        with tm.phase("Scan"):
            adv, ret, stats = gae_scan_tm(rew, done, self.val, self.gamma, self.lam, adv=self.adv, ret=self.ret,
                                          stats_part=self.stats_part, stats_out=self.adv_stats,
                                          tval=self.tval if tobs is not None else None)
            if not rew.is_cuda:
                self.adv.view(-1).copy_(adv.reshape(-1))
                self.ret.view(-1).copy_(ret.reshape(-1))
                self.adv_stats.copy_(stats)
            self.comm.all_reduce_sum_(self.adv_stats)
        inv_B = 1.0 / (B * self.comm.world)
        discrete = lr.discrete
        a = act.reshape(B) if discrete else None
        ac = None if discrete else act.reshape(B, -1)
        m = None if mask is None else mask.reshape(B, -1)
        with tm.phase("Optimize"):
            lr.optimize(obs_b, act=a, actc=ac, mask=m, adv=self.adv.view(-1), ret=self.ret.view(-1),
                        adv_stats=self.adv_stats, logp_old=logp.reshape(-1), inv_B=inv_B)


def episode_metrics(comm: Comm, n, s, sq, mx, mn, sum_len) -> dict:
    dev = "cuda" if comm.backend == "nccl" else "cpu"
    vec = torch.tensor([n, s, sq, sum_len], dtype=torch.float64, device=dev)
    comm.all_reduce_sum_(vec)
    mxt = torch.tensor([mx], dtype=torch.float64, device=dev)
    mnt = torch.tensor([mn], dtype=torch.float64, device=dev)
    comm.all_reduce_max_(mxt)
    comm.all_reduce_min_(mnt)
    n, s, sq, sl = vec.tolist()
    if n <= 0:
        nan = float("nan")
        return {"AverageEpRet": nan, "StdEpRet": nan, "MaxEpRet": nan, "MinEpRet": nan, "EpLen": nan, "Episodes": 0}
    mean = s / n
    return {"AverageEpRet": mean, "StdEpRet": math.sqrt(max(sq / n - mean * mean, 0.0)), "MaxEpRet": mxt.item(),
            "MinEpRet": mnt.item(), "EpLen": sl / n, "Episodes": int(n)}
