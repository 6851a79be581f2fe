"""Policy-gradient learner over flat device batches (REINFORCE, A2C, PPO).

Shared by the trajectory-fed plugin algorithms (reinforce.py / ppo.py / a2c.py) and by
the vectorised on-device trainer.  Every optimisation step is one fused fwd+bwd HIP
launch + one fused reduce+Adam launch (+ one RCCL all-reduce with several ranks):

  REINFORCE (REINFORCE.py:97-125): 1 policy step on -mean(logp * adv) then
            ``train_vf_iters`` value steps (separate optimisers -- the reference's
            pi_optimizer also covered the baseline parameters, defect A15);
  A2C      : 1 policy step with an entropy bonus + value steps;
  PPO      : ``train_pi_iters`` clipped-surrogate epochs with approximate-KL early
            stopping, then ``train_vf_iters`` value epochs.  With ``num_minibatches`` M > 1
            every epoch reshuffles the batch (one device ``randperm`` per epoch) and takes M
            steps on disjoint minibatches (the usual PPO schedule); advantages keep the
            full-batch normalisation statistics.  M = 1 is the full-batch form, whose value
            loop is one hipGraph replay.

hipGraphs: with ``use_graphs`` on a GPU the WHOLE epoch of updates (policy step(s) + the
value loop, with their RCCL all-reduces at world > 1) is captured once per input-buffer set
and replayed -- the multi-rank epoch is one replay instead of ~4 x (1 + train_vf_iters)
eager launches.  Not capturable (eager, value loop still a graph): PPO with target_kl (its
early stop reads the KL on the host), minibatches (a fresh permutation per epoch), gloo.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import GradHead, MLPSpec, mlp_grad, grad_slabs
from ..parallel.comm import Comm
from ..utils.tracing import gc_paused
from .core import FlatNet, ValueLoop, _muted


class PGLearner:
    def __init__(self, algo: str, obs_dim: int, act_dim: int, hidden: int = 128, discrete: bool = True,
                 with_baseline: bool = True, pi_lr: float = 3e-4, vf_lr: float = 1e-3, train_vf_iters: int = 80,
                 train_pi_iters: int = 1, clip_ratio: float = 0.2, target_kl: Optional[float] = None,
                 ent_coef: float = 0.0, device="cpu", seed: int = 0, comm: Optional[Comm] = None,
                 use_graphs: bool = True, log_std_init: float = -0.5, pi_params=None, vf_params=None,
                 num_minibatches: int = 1):
        algo = algo.lower()
        assert algo in ("reinforce", "a2c", "ppo"), algo
        self.algo = algo
        self.obs_dim, self.act_dim, self.hidden = obs_dim, act_dim, hidden
        self.discrete = discrete
        self.with_baseline = with_baseline or algo in ("a2c", "ppo")
        self.train_vf_iters = int(train_vf_iters)
        self.train_pi_iters = int(train_pi_iters) if algo == "ppo" else 1
        self.clip_ratio = float(clip_ratio)
        self.target_kl = target_kl
        self.ent_coef = float(ent_coef)
        self.device = torch.device(device)
        self.comm = comm or Comm()
        g = torch.Generator().manual_seed(int(seed))
        self.pi = FlatNet(MLPSpec(obs_dim, hidden, act_dim, not discrete), pi_lr, self.device, g, params=pi_params,
                          log_std_init=log_std_init)
        self.vf = FlatNet(MLPSpec(obs_dim, hidden, 1), vf_lr, self.device, g, params=vf_params) \
            if self.with_baseline else None
        self.vloop = ValueLoop(self.vf, self.comm, use_graph=use_graphs) if self.vf is not None else None
        self.num_minibatches = max(1, int(num_minibatches)) if algo == "ppo" else 1
        # minibatch shuffles: one stream per rank (different data shards), reproducible from the seed
        self.mb_seed = int(seed) * 1000003 + 17 + self.comm.rank
        self._mb_gen = torch.Generator(device=self.device).manual_seed(self.mb_seed) \
            if self.num_minibatches > 1 else None
        self._pi_slab = None
        self._pi_loss = None
        self.last = {}
        self.use_graphs = bool(use_graphs)
        self.graphs_enabled = True  # toggled off for epochs with a changing batch (agent rows)
        self.before_capture = None  # quiesce helper threads that issue HIP calls (host_trainer)
        self._opt_graphs = {}
        self.graph_replays = 0

    @property
    def head(self) -> int:
        if self.algo == "ppo":
            return int(GradHead.PPO_CAT if self.discrete else GradHead.PPO_GAUSS)
        return int(GradHead.PG_CAT if self.discrete else GradHead.PG_GAUSS)

    def _slabs(self, B):
        if self.device.type != "cuda":
            return None, None
        ns = grad_slabs(B, self.device)
        if self._pi_slab is None or self._pi_slab.shape[0] < ns:
            # (captured graphs keep the old slab alive through their entries)
            self._pi_slab = torch.empty(ns, self.pi.P, device=self.device)
            self._pi_loss = torch.empty(ns, 8, device=self.device)
        return self._pi_slab[:ns], self._pi_loss[:ns]

    def capturable(self) -> bool:
        """The whole optimize() epoch can be one hipGraph."""
        return (self.use_graphs and self.graphs_enabled and self.device.type == "cuda" and self.comm.graph_safe
                and self.num_minibatches == 1 and not (self.algo == "ppo" and self.target_kl is not None))

    def optimize(self, obs, act=None, actc=None, mask=None, adv=None, ret=None, adv_stats=None, logp_old=None,
                 inv_B: Optional[float] = None, nvalid=None, inv_B_dev=None):
        """One epoch of updates on a prepared batch (adv/ret already computed).

        ``nvalid`` / ``inv_B_dev`` (device scalars, grad_args.h): only the first nvalid rows
        count and the loss scale is read from memory -- a padded batch whose valid row count
        changes every epoch (agent rows, rollout_learn.py) replays ONE captured graph.

        Returns a dict of *device* tensors (loss slabs) -- call ``summarize`` to sync.
        """
        B = obs.shape[0]
        if inv_B is None:
            inv_B = 1.0 / max(B * self.comm.world, 1)
        if self.capturable():
            return self._optimize_graph(obs, act, actc, mask, adv, ret, adv_stats, logp_old, float(inv_B), nvalid,
                                        inv_B_dev)
        if (nvalid is not None or inv_B_dev is not None) and self.num_minibatches > 1:
            raise ValueError("a device-side row count needs the full-batch schedule (num_minibatches 1)")
        return self._optimize_eager(obs, act, actc, mask, adv, ret, adv_stats, logp_old, inv_B, nvalid, inv_B_dev)

    def _nets(self):
        return [n for n in (self.pi, self.vf) if n is not None]

    def _optimize_graph(self, obs, act, actc, mask, adv, ret, adv_stats, logp_old, inv_B: float, nvalid=None,
                        inv_B_dev=None):
        """Capture (once per input-buffer set) and replay the whole epoch of updates."""
        B = obs.shape[0]
        args = (obs, act, actc, mask, adv, ret, adv_stats, logp_old, nvalid, inv_B_dev)
        key = (B, inv_B) + tuple(0 if t is None else t.data_ptr() for t in args)
        ent = self._opt_graphs.get(key)
        if ent is None:
            if len(self._opt_graphs) >= 4:
                self._opt_graphs.clear()
            self._slabs(B)
            if self.vloop is not None:
                self.vloop.prepare(B, self.train_vf_iters, inv_B, self.device)
            if self.before_capture is not None:
                self.before_capture()
            nets = self._nets()
            v0 = [n.version for n in nets]
            state = [t.clone() for n in nets for t in (n.params, n.m, n.v, n.step)]
            # warm up eagerly once on the real buffers (kernel attributes, allocator), then
            # restore the optimiser state so the warm-up leaves no trace.  The warm-up's
            # collectives are muted (Comm.muted): whether this rank captures now is a rank-local
            # decision (its own input buffers / agent rows / cache), so a real all-reduce here
            # would pair with another rank's unrelated calls.  The RCCL communicator
            # already exists: the statistics all-reduce of the same epoch ran before this.
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s), _muted(self.comm):
                self._optimize_body(*args, inv_B=inv_B, vf_iters=min(1, self.train_vf_iters))
            torch.cuda.current_stream(self.device).wait_stream(s)
            it = iter(state)
            for n in nets:
                for t in (n.params, n.m, n.v, n.step):
                    t.copy_(next(it))
            for n, v in zip(nets, v0):
                n.version = v
            g = torch.cuda.CUDAGraph()
            # thread_local: a host rollout thread (host_trainer overlap) may issue HIP calls meanwhile
            with gc_paused(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                last = self._optimize_body(*args, inv_B=inv_B, vf_iters=self.train_vf_iters)
            dv = [n.version - v for n, v in zip(nets, v0)]
            for n, v in zip(nets, v0):
                n.version = v
            # the entry holds every buffer the graph reads or writes: a later capture for another
            # batch shape selects / grows other buffers, and these must not be freed (and reused
            # by the caching allocator) under this graph
            keep = (self._pi_slab, self._pi_loss, self.vloop.bufs if self.vloop is not None else None)
            ent = (g, dict(last), dv, keep)
            self._opt_graphs[key] = ent
        g, last, dv, keep = ent
        if keep[2] is not None:
            self.vloop.use_bufs(*keep[2])  # summarize() reads this graph's value-loss slabs
        g.replay()
        self.graph_replays += 1
        for n, d in zip(self._nets(), dv):
            n.version += d
        self.last = dict(last)
        return self.last

    def _optimize_body(self, obs, act, actc, mask, adv, ret, adv_stats, logp_old, nvalid=None, inv_B_dev=None, *,
                       inv_B: float, vf_iters: int):
        """Full-batch epoch (no host reads): the capturable form of _optimize_eager."""
        H, A = self.hidden, self.act_dim
        slab, ls = self._slabs(obs.shape[0])
        pi_loss = None
        for it in range(self.train_pi_iters):
            out = mlp_grad(self.head, self.pi.params, obs, A, H, mask=mask, act=act, actc=actc, adv=adv,
                           logp_old=logp_old, adv_stats=adv_stats, inv_B=inv_B, clip_eps=self.clip_ratio,
                           ent_coef=self.ent_coef, grad_slab=slab, loss_slab=ls, nvalid=nvalid, inv_B_dev=inv_B_dev)
            if it == 0:
                # one policy step: its loss slab stays untouched until the next epoch, so
                # summarize() sums it when (if) the statistics are read -- no reduction launch
                # inside every epoch (~11 us of a 2 ms reference-hyperparameter epoch)
                pi_loss = out[1] if self.train_pi_iters == 1 else out[1].sum(0)
            self.pi.apply(out[0], self.comm)
        if self.vloop is not None and vf_iters > 0:
            self.vloop.run_body(obs, ret, vf_iters, inv_B, nvalid, inv_B_dev)
        return {"pi_loss": pi_loss, "kl_stop": None}

    def _optimize_eager(self, obs, act, actc, mask, adv, ret, adv_stats, logp_old, inv_B, nvalid=None,
                        inv_B_dev=None):
        B = obs.shape[0]
        H, A = self.hidden, self.act_dim
        M = self.num_minibatches
        slab, ls = self._slabs(B)
        kl_stop = None
        pi_loss = None
        step = 0
        for it in range(self.train_pi_iters):
            if M == 1:
                batches = [(None, inv_B)]
            else:
                batches = [(idx, inv_B * B / idx.numel()) for idx in self.minibatches(B)]
            for idx, inv in batches:
                def sel(t):
                    return t if idx is None or t is None else t.index_select(0, idx)

                out = mlp_grad(self.head, self.pi.params, sel(obs), A, H, mask=sel(mask), act=sel(act),
                               actc=sel(actc), adv=sel(adv), logp_old=sel(logp_old), adv_stats=adv_stats, inv_B=inv,
                               clip_eps=self.clip_ratio, ent_coef=self.ent_coef, grad_slab=slab, loss_slab=ls,
                               nvalid=nvalid, inv_B_dev=inv_B_dev)
                if step == 0:
                    pi_loss = out[1] if (self.train_pi_iters == 1 and M == 1) else out[1].sum(0).clone()
                if self.algo == "ppo" and self.target_kl is not None and step > 0:
                    # approx KL of the current policy (measured in this step's forward)
                    st = out[1].sum(0)
                    st = self.comm.all_reduce_sum_(st.clone())
                    kl = (st[2] / torch.clamp(st[5], min=1.0)).item()
                    if kl > 1.5 * self.target_kl:
                        kl_stop = it
                        break
                self.pi.apply(out[0], self.comm)
                step += 1
            if kl_stop is not None:
                break
        if self.vloop is not None and self.train_vf_iters > 0:
            if M == 1:
                self.vloop.run(obs, ret, self.train_vf_iters, inv_B, nvalid, inv_B_dev)
            else:
                for ep in range(self.train_vf_iters):
                    for j, idx in enumerate(self.minibatches(B)):
                        self.vloop.step(obs.index_select(0, idx), ret.index_select(0, idx), inv_B * B / idx.numel(),
                                        first=(ep == 0 and j == 0))
        self.last = {"pi_loss": pi_loss, "kl_stop": kl_stop}
        return self.last

    def minibatches(self, B: int):
        """Row indices of one epoch's ``num_minibatches`` disjoint minibatches (a fresh
        permutation of the B rows; sizes differ by at most one row)."""
        M = self.num_minibatches
        perm = torch.randperm(B, device=self.device, generator=self._mb_gen)
        return [perm[i * B // M:(i + 1) * B // M] for i in range(M)]

    def summarize(self) -> dict:
        """Synchronising read of the last optimize() statistics (global over ranks)."""
        out = {}
        pl = self.last.get("pi_loss")
        if pl is not None:
            pl = pl.sum(0) if pl.dim() == 2 else pl.clone()  # [slabs, 8] loss slab or its sum
            v = self.comm.all_reduce_sum_(pl.to(self.device)).tolist()
            n = max(v[5], 1.0)
            out.update(LossPi=v[0] / n, Entropy=v[1] / n, KL=v[2] / n, ClipFrac=v[3] / n, DeltaLossPi=0.0)
        if self.vloop is not None and self.vloop.loss_last is not None:
            l1 = self.vloop.loss_last.sum(0)
            l0 = self.vloop.loss_first.sum(0)
            v = self.comm.all_reduce_sum_(torch.stack([l1[0], l1[4], l1[5], l0[0]]).to(self.device)).tolist()
            n = max(v[2], 1.0)
            out.update(LossV=v[0] / n, VVals=v[1] / n, DeltaLossV=(v[0] - v[3]) / n)
        if self.last.get("kl_stop") is not None:
            out["StopIter"] = self.last["kl_stop"]
        return out

    def state_tensors(self):
        """The live tensors that ARE this learner's state (parameters, Adam moments, device
        step counters): the elastic epoch-start snapshot copies these on the device."""
        return [t for n in self._nets() for t in (n.params, n.m, n.v, n.step)]

    def drop_graphs(self):
        """Forget every captured graph (after a process-group re-form their RCCL collectives
        belong to a destroyed communicator and must never replay)."""
        self._opt_graphs.clear()
        if self.vloop is not None:
            self.vloop._graphs.clear()

    def broadcast_state_(self, comm: Comm, src: int = 0):
        """Overwrite this learner's parameters and Adam state with rank ``src``'s (after an
        elastic re-form a new learner may join without state)."""
        for net in (self.pi, self.vf):
            if net is None:
                continue
            for t in (net.params, net.m, net.v, net.step):
                comm.broadcast_(t, src)

    def state_dict(self) -> dict:
        sd = {"pi": self.pi.state_dict()}
        if self.vf is not None:
            sd["vf"] = self.vf.state_dict()
        return sd

    def load_state_dict(self, sd: dict):
        self.pi.load_state_dict(sd["pi"])
        if self.vf is not None and "vf" in sd:
            self.vf.load_state_dict(sd["vf"])
