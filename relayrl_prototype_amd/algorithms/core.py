"""Device learner building blocks shared by REINFORCE / A2C / PPO.

``FlatNet`` = one MLP as a single flat fp32 parameter vector + fused-Adam state (m, v,
device step counter).  Gradients come out of the fused fwd+bwd kernel as per-workgroup
slabs; with one rank the slabs feed the fused reduce+Adam kernel directly, with several
ranks (``Comm.multi``) they are reduced to one flat vector, all-reduced over RCCL, then Adam
runs on it.  Both forms are captured into hipGraphs: RCCL collectives replay inside a graph,
so the multi-rank value loop is one replay per epoch too (``Comm.graph_safe``).
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import MLPSpec, GradHead, adam_step, mlp_grad, reduce_slabs, grad_slabs
from ..parallel.comm import Comm
from ..utils.faults import maybe_stall_at
from ..utils.tracing import gc_paused


class FlatNet:
    def __init__(self, spec: MLPSpec, lr: float, device, generator: Optional[torch.Generator] = None,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, params: Optional[torch.Tensor] = None,
                 log_std_init: float = -0.5):
        self.spec = spec
        self.device = torch.device(device)
        self.lr = float(lr)
        self.betas = betas
        self.eps = float(eps)
        self.weight_decay = float(weight_decay)
        if params is None:
            params = spec.init(generator, log_std_init=log_std_init)
        assert params.numel() == spec.P, (params.numel(), spec.P)
        self.params = params.detach().float().contiguous().to(self.device).clone()
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.step = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.ticket = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.grad = torch.zeros_like(self.params)
        self.version = 0

    @property
    def P(self) -> int:
        return self.spec.P

    def apply(self, slab: torch.Tensor, comm: Optional[Comm] = None, step_add: int = 0, step_inc: int = 1):
        """Reduce the gradient slabs (and all-reduce across ranks) then take one Adam step
        (``step_add`` / ``step_inc``: see ops.adam_step, the loop form of the step counter)."""
        b1, b2 = self.betas
        if comm is None or not comm.multi:
            adam_step(self.params, self.m, self.v, self.step, self.ticket, self.lr, slab=slab, beta1=b1, beta2=b2,
                      eps=self.eps, weight_decay=self.weight_decay, step_add=step_add, step_inc=step_inc)
        else:
            reduce_slabs(slab, 1.0, out=self.grad)
            comm.all_reduce_sum_(self.grad)
            adam_step(self.params, self.m, self.v, self.step, self.ticket, self.lr, grad=self.grad, beta1=b1,
                      beta2=b2, eps=self.eps, weight_decay=self.weight_decay, step_add=step_add, step_inc=step_inc)
        self.version += 1

    def state_dict(self) -> dict:
        return {"params": self.params.detach().cpu(), "m": self.m.cpu(), "v": self.v.cpu(),
                "step": self.step.cpu(), "lr": torch.tensor(self.lr)}

    def load_state_dict(self, sd: dict):
        self.params.copy_(sd["params"].to(self.device))
        self.m.copy_(sd["m"].to(self.device))
        self.v.copy_(sd["v"].to(self.device))
        self.step.copy_(sd["step"].to(self.device))
        if "lr" in sd:
            self.lr = float(sd["lr"])


class ValueLoop:
    """``iters`` x (fused value fwd+bwd -> fused reduce+Adam), optionally captured into one
    hipGraph (REINFORCE.py:110-115 runs this loop 80 times per epoch)."""

    def __init__(self, net: FlatNet, comm: Optional[Comm], use_graph: bool = True):
        self.net = net
        self.comm = comm
        # with several ranks the loop's all-reduces are captured too (RCCL on the device); a
        # gloo group issues host calls, which a graph cannot hold
        self.use_graph = use_graph and net.device.type == "cuda" and (comm is None or comm.graph_safe)
        self._graphs = {}
        self._bufs = {}  # shape key -> (slab, loss_first, loss_last): captured graphs keep theirs
        self._key = None
        self._slab = None
        self.loss_first = None
        self.loss_last = None
        # called before a graph capture starts: a trainer whose helper thread issues HIP calls
        # (host_trainer's overlapped rollout) quiesces it here -- HIP invalidates a capture when
        # another thread synchronises on the device meanwhile, whatever that thread's mode
        self.before_capture = None

    def _body(self, obs, ret, iters, inv_B, slab, ls_first, ls_last, nvalid=None, inv_B_dev=None):
        H = self.net.spec.H
        hook = not torch.cuda.is_current_stream_capturing()
        for k in range(iters):
            if hook:
                maybe_stall_at("viter", k)
            ls = ls_first if k == 0 else ls_last
            mlp_grad(GradHead.VALUE_MSE, self.net.params, obs, 1, H, ret=ret, inv_B=inv_B, grad_slab=slab,
                     loss_slab=ls, nvalid=nvalid, inv_B_dev=inv_B_dev)
            # Adam step s0 + k + 1; only the last update of the loop advances the counter (by iters)
            self.net.apply(slab, self.comm, step_add=k, step_inc=iters if k == iters - 1 else 0)

    def step(self, obs: torch.Tensor, ret: torch.Tensor, inv_B: float, first: bool = False):
        """One eager value step on a (mini)batch; ``first`` marks the step whose loss is
        reported as the epoch's starting loss (PPO minibatch schedule, learner.py)."""
        dev = obs.device
        slab = ls = None
        if dev.type == "cuda":
            ns = grad_slabs(obs.shape[0], dev)
            if getattr(self, "_mb_slab", None) is None or self._mb_slab.shape[0] < ns:
                self._mb_slab = torch.empty(ns, self.net.P, device=dev)
                self._mb_loss = torch.empty(ns, 8, device=dev)
            slab, ls = self._mb_slab, self._mb_loss
        g, ls = mlp_grad(GradHead.VALUE_MSE, self.net.params, obs, 1, self.net.spec.H, ret=ret, inv_B=inv_B,
                         grad_slab=slab, loss_slab=ls)
        if first:
            self.loss_first = ls.clone()
        self.loss_last = ls
        self.net.apply(g, self.comm)

    def prepare(self, B: int, iters: int, inv_B: float, dev) -> None:
        """Select (allocating once per shape) the slab / loss buffers of this batch shape
        (before any capture).  Buffers are never reallocated under a graph that uses them:
        each shape keeps its own set, and every graph entry holds a reference to the set it
        was captured with (a padded agent-row batch used to free the buffers of
        the unpadded batch's graph)."""
        shape_key = (B, iters, float(inv_B))
        if self._key != shape_key:
            bufs = self._bufs.get(shape_key)
            if bufs is None:
                if len(self._bufs) >= 8:
                    self._bufs.clear()  # graphs still hold theirs
                ns = grad_slabs(B, dev)
                bufs = (torch.empty(ns, self.net.P, device=dev), torch.zeros(ns, 8, device=dev),
                        torch.zeros(ns, 8, device=dev))
                self._bufs[shape_key] = bufs
            self.use_bufs(shape_key, bufs)

    def use_bufs(self, shape_key, bufs) -> None:
        self._key = shape_key
        self._slab, self.loss_first, self.loss_last = bufs

    @property
    def bufs(self):
        return self._key, (self._slab, self.loss_first, self.loss_last)

    def run_body(self, obs: torch.Tensor, ret: torch.Tensor, iters: int, inv_B: float, nvalid=None,
                 inv_B_dev=None):
        """The loop's launches on the current stream (inside an enclosing capture, e.g.
        PGLearner's whole-optimize graph); ``prepare`` must have run."""
        self._body(obs, ret, iters, inv_B, self._slab, self.loss_first, self.loss_last, nvalid, inv_B_dev)

    def run(self, obs: torch.Tensor, ret: torch.Tensor, iters: int, inv_B: float, nvalid=None, inv_B_dev=None):
        B = obs.shape[0]
        dev = obs.device
        if iters <= 0:
            return
        if dev.type != "cuda":
            # CPU oracle path: autograd + torch Adam math
            for k in range(iters):
                maybe_stall_at("viter", k)
                g, ls = mlp_grad(GradHead.VALUE_MSE, self.net.params, obs, 1, self.net.spec.H, ret=ret, inv_B=inv_B,
                                 nvalid=nvalid, inv_B_dev=inv_B_dev)
                if k == 0:
                    self.loss_first = ls
                self.loss_last = ls
                self.net.apply(g, self.comm)
            return
        self.prepare(B, iters, inv_B, dev)
        if not self.use_graph:
            self._body(obs, ret, iters, inv_B, self._slab, self.loss_first, self.loss_last, nvalid, inv_B_dev)
            return
        v0 = self.net.version
        # one graph per input buffer set (double-buffered trainers, padded agent-row batches)
        # and batch shape; the entry keeps the buffers it was captured with
        gkey = (obs.data_ptr(), ret.data_ptr(), 0 if nvalid is None else nvalid.data_ptr(),
                0 if inv_B_dev is None else inv_B_dev.data_ptr(), self._key)
        ent = self._graphs.get(gkey)
        if ent is None:
            if len(self._graphs) >= 4:
                self._graphs.clear()
            if self.before_capture is not None:
                self.before_capture()
            # Warm up once eagerly (kernel attributes, allocator) on the real buffers, with the
            # collectives muted (rank-local, Comm.muted), then restore the optimiser state so
            # the warm-up step leaves no trace.
            saved = [t.clone() for t in (self.net.params, self.net.m, self.net.v, self.net.step)]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s), _muted(self.comm):
                self._body(obs, ret, 1, inv_B, self._slab, self.loss_first, self.loss_last, nvalid, inv_B_dev)
            torch.cuda.current_stream().wait_stream(s)
            for dst, src in zip((self.net.params, self.net.m, self.net.v, self.net.step), saved):
                dst.copy_(src)
            g = torch.cuda.CUDAGraph()
            # thread_local: a host rollout thread (host_trainer overlap) may issue HIP calls meanwhile
            with gc_paused(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                self._body(obs, ret, iters, inv_B, self._slab, self.loss_first, self.loss_last, nvalid, inv_B_dev)
            ent = (g, self.bufs)
            self._graphs[gkey] = ent
        g, (key, bufs) = ent
        self.use_bufs(key, bufs)
        g.replay()
        self.net.version = v0 + iters


def _muted(comm: Optional[Comm]):
    """comm.muted() (no collectives), or a no-op context without a comm."""
    import contextlib

    return comm.muted() if comm is not None else contextlib.nullcontext()
