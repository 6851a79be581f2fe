"""Shared "rollout -> returns -> optimise" step for the vectorised trainers."""
from __future__ import annotations

import math
from typing import Optional

import torch

from ..algorithms.learner import PGLearner
from ..ops import FwdMode, gae_scan_tm, mlp_forward, scan_flat
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
        # agent uploads folded into the next batch (runtime/engine.py): a FlatBuffer.take() dict
        self.pending_rows = None
        self.last_agent_rows = 0
        # several ranks with uploads staged on one of them (runtime/engine.py): agree on the
        # global row count each epoch (see learn; the fallback of the padded path below)
        self.count_sync = False
        # agent rows on a capturable learner: ONE padded batch [B + agent_cap] whose valid row
        # count (nvalid) and loss scale (1 / global rows, from the all-reduced statistics) live
        # on the device, so epochs with uploads replay a captured graph too
        self.agent_rows_enabled = False
        self.agent_cap = 0
        self._pad = None
        self._nvalid = None
        self._inv_dev = None
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
            extra, self.pending_rows = self.pending_rows, None
            self.last_agent_rows = 0
            folded = None
            if extra is not None and extra["obs"].shape[0] > 0:
                # the uploads' scan runs BEFORE the statistics all-reduce: their advantage sums
                # and row count enter the global normalisation on every rank
                with tm.phase("AgentRows"):
                    folded = self._fold_scan(extra)
            self.comm.all_reduce_sum_(self.adv_stats)
        discrete = lr.discrete
        a = act.reshape(B) if discrete else None
        ac = None if discrete else act.reshape(B, -1)
        m = None if mask is None else mask.reshape(B, -1)
        adv_b, ret_b, logp_b = self.adv.view(-1), self.ret.view(-1), logp.reshape(-1)
        B = obs_b.shape[0]
        any_rows = self.last_agent_rows > 0
        if self._device_shape_ok(folded):
            self._optimize_padded(folded, obs_b, a, ac, m, adv_b, ret_b, logp_b)
            return
        if folded is not None:
            obs_b, a, ac, m, adv_b, ret_b, logp_b = self._fold_cat(folded, obs_b, a, ac, m, adv_b, ret_b, logp_b)
            B = obs_b.shape[0]
            any_rows = True
        if self.count_sync:
            # several ranks, uploads staged on rank 0 only: the global row count (all-reduced
            # statistics) sets the loss scale on every rank, and every rank goes eager when
            # any rank folded rows (one host read per epoch, only in this mode)
            total = int(round(float(self.adv_stats[2].item())))
            inv_B = 1.0 / max(total, 1)
            any_rows = total != self.T * self.N * self.K * self.comm.world
        else:
            inv_B = 1.0 / (B * self.comm.world)
        graphs = lr.vloop.use_graph if lr.vloop is not None else False
        if any_rows:
            # a new batch shape every epoch: no graph capture
            lr.graphs_enabled = False
            if lr.vloop is not None:
                lr.vloop.use_graph = False
        try:
            with tm.phase("Optimize"):
                lr.optimize(obs_b, act=a, actc=ac, mask=m, adv=adv_b, ret=ret_b, adv_stats=self.adv_stats,
                            logp_old=logp_b, inv_B=inv_B)
        finally:
            lr.graphs_enabled = True
            if lr.vloop is not None:
                lr.vloop.use_graph = graphs

    def _fold_scan(self, d):
        """Agent uploads (concatenated paths, FlatBuffer.take): their own flat segmented scan
        (finish_path semantics, REINFORCE.py:70-95 / replay_buffer.py:48-79) with V(s) from the
        current value net and V(s_T) bootstraps for cut paths; their advantage sums are added to
        this rank's batch statistics (before the all-reduce)."""
        lr = self.learner
        H = lr.hidden
        dev = self.adv_stats.device
        obs_e = d["obs"].to(dev)
        boot = d["boot"]
        val = None
        if lr.vf is not None:
            val = mlp_forward(FwdMode.VALUE, lr.vf.params, obs_e, 1, H)["v"]
            boot = torch.where(torch.isnan(boot), val, boot)  # cut path without s_T: V(s_last)
            bi = d["boot_idx"]
            if bi.numel():
                vb = mlp_forward(FwdMode.VALUE, lr.vf.params, d["boot_obs"], 1, H)["v"]
                boot = boot.index_copy(0, bi.to(boot.device), vb.to(boot.dtype))
        else:
            boot = torch.zeros_like(boot)  # no value net: last_val dropped (replay_buffer.py:74-77)
        adv_e, ret_e, st_e = scan_flat(d["rew"], d["done"], val, boot, self.gamma, self.lam)
        self.adv_stats.add_(st_e.to(dev))
        if d["has_logp"]:
            logp_e = d["logp"]
        else:  # uploads without log-probs: the current policy's (PPO ratio 1 on those rows)
            mode = FwdMode.CAT_EVAL if lr.discrete else FwdMode.GAUSS_EVAL
            logp_e = mlp_forward(mode, lr.pi.params, obs_e, lr.act_dim, H, mask=d["mask"],
                                 act_in=d["act"] if lr.discrete else None,
                                 actc_in=None if lr.discrete else d["act"])["logp"]
        return dict(d, obs=obs_e, adv=adv_e, ret=ret_e, logp=logp_e)

    # ------------------------------------------------------------------ padded agent rows
    def _device_shape_ok(self, folded) -> bool:
        """Agent rows enabled, a capturable learner on the GPU, and this epoch's uploads (if
        any) fit the padded capacity."""
        lr = self.learner
        if not (self.agent_rows_enabled and self.agent_cap > 0 and lr.device.type == "cuda" and lr.capturable()):
            return False
        return folded is None or folded["obs"].shape[0] <= self.agent_cap

    def _pad_buffers(self, B, D, A, dev):
        lr = self.learner
        C = self.agent_cap
        cap = B + C
        p = {"obs": torch.zeros(cap, D, device=dev), "adv": torch.zeros(cap, device=dev),
             "ret": torch.zeros(cap, device=dev), "logp": torch.zeros(cap, device=dev),
             "mask": torch.ones(cap, A, device=dev) if lr.discrete else None}
        p["act"] = torch.zeros(cap, dtype=torch.int32, device=dev) if lr.discrete else torch.zeros(cap, A, device=dev)
        self._pad = p
        self._nvalid = torch.zeros(1, dtype=torch.int32, device=dev)
        return p

    def _optimize_padded(self, folded, obs_b, a, ac, m, adv_b, ret_b, logp_b):
        """Replayable epoch: the loss scale 1 / (global rows) is computed on the device from the
        all-reduced statistics (identical on every rank); with uploads, the batch and the rows are
        copied into the padded buffers and only the first nvalid rows count."""
        lr = self.learner
        dev = lr.device
        B = obs_b.shape[0]
        if folded is None and not self.comm.multi:
            # one rank, no uploads: the host scale 1 / B is exact (no device scalar needed)
            with self.timer.phase("Optimize"):
                lr.optimize(obs_b, act=a, actc=ac, mask=m, adv=adv_b, ret=ret_b, adv_stats=self.adv_stats,
                            logp_old=logp_b, inv_B=1.0 / B)
            return
        if self._inv_dev is None:
            self._inv_dev = torch.zeros(1, device=dev)
        torch.reciprocal(self.adv_stats[2:3], out=self._inv_dev)
        with self.timer.phase("Optimize"):
            if folded is None:
                lr.optimize(obs_b, act=a, actc=ac, mask=m, adv=adv_b, ret=ret_b, adv_stats=self.adv_stats,
                            logp_old=logp_b, inv_B=1.0 / (B * self.comm.world), inv_B_dev=self._inv_dev)
                return
            n = folded["obs"].shape[0]
            D = obs_b.shape[1]
            A = lr.act_dim
            p = self._pad
            if p is None or p["obs"].shape[0] != B + self.agent_cap or p["obs"].shape[1] != D:
                p = self._pad_buffers(B, D, A, dev)
            p["obs"][:B].copy_(obs_b)
            p["obs"][B:B + n].copy_(folded["obs"])
            for k, main, up in (("adv", adv_b, folded["adv"]), ("ret", ret_b, folded["ret"]),
                                ("logp", logp_b, folded["logp"].reshape(-1))):
                p[k][:B].copy_(main)
                p[k][B:B + n].copy_(up)
            if lr.discrete:
                p["act"][:B].copy_(a)
                p["act"][B:B + n].copy_(folded["act"].reshape(-1).to(torch.int32))
            else:
                p["act"][:B].copy_(ac)
                p["act"][B:B + n].copy_(folded["act"].reshape(n, -1))
            use_mask = lr.discrete and (m is not None or not folded.get("mask_trivial", False))
            if use_mask:
                if m is not None:
                    p["mask"][:B].copy_(m)
                else:
                    p["mask"][:B].fill_(1.0)
                p["mask"][B:B + n].copy_(folded["mask"])
            self._nvalid.fill_(B + n)
            self.last_agent_rows = n
            lr.optimize(p["obs"], act=p["act"] if lr.discrete else None, actc=None if lr.discrete else p["act"],
                        mask=p["mask"] if use_mask else None, adv=p["adv"], ret=p["ret"], adv_stats=self.adv_stats,
                        logp_old=p["logp"], inv_B=1.0 / ((B + self.agent_cap) * self.comm.world), nvalid=self._nvalid,
                        inv_B_dev=self._inv_dev)

    def _fold_cat(self, e, obs_b, a, ac, m, adv_b, ret_b, logp_b):
        """The scanned uploads appended to the device batch as extra rows: one concatenated
        batch for the policy and value steps."""
        lr = self.learner
        n = e["obs"].shape[0]
        cat = torch.cat
        obs_c = cat([obs_b, e["obs"]])
        if lr.discrete:
            a = cat([a, e["act"].to(a.dtype)])
        else:
            ac = cat([ac, e["act"].reshape(n, -1)])
        mask_e = e["mask"]
        if m is not None or (lr.discrete and not bool((mask_e == 1).all())):
            m_b = m if m is not None else torch.ones(obs_b.shape[0], lr.act_dim, device=obs_b.device)
            m = cat([m_b, mask_e])
        self.last_agent_rows = n
        return (obs_c, a, ac, m, cat([adv_b, e["adv"]]), cat([ret_b, e["ret"]]),
                cat([logp_b, e["logp"].reshape(-1)]))


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
