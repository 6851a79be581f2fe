"""Process-group communicator: one process per GPU, RCCL over xGMI ("nccl" backend on
ROCm), gloo for CPU tests.

The reference has no collectives at all: trajectories fan in over
ZMQ/gRPC and TorchScript files fan out.  Here every data-plane exchange is a
collective on ONE flat buffer:

* C8 gradient sync     -> ``all_reduce_sum_`` of the flat fp32 gradient (one call per update)
* C2 weight fan-out    -> ``broadcast_`` of the flat fp32 parameter vector from the learner
* C1 rollout fan-in    -> ``gather_to`` (paired send/recv so each actor uses its own link)
* advantage statistics -> ``all_reduce_sum_`` of a 3-float vector

xGMI is point-to-point (7 links per GPU); the flat gradient of a 128x128 MLP is ~70 KB,
so these are latency-bound: keep them fused, one call per optimiser step -- and capture the
optimiser loops WITH their all-reduces into hipGraphs (RCCL collectives replay inside a
graph), so a world > 1 epoch is not 80 x 4 eager launches.

``RRL_FORCE_COLLECTIVES=1`` sends a ONE-rank process group through the world > 1 code path
(``Comm.multi``): slab reduce -> real ``dist.all_reduce`` -> Adam, bucketed DP all-reduces,
captured graphs.  A one-GPU box cannot host two RCCL ranks, so this is how the multi-rank
path's RCCL calls (and their graph capture) are exercised and timed on one MI355X.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist


def dist_env() -> tuple:
    """(rank, local_rank, world) from torchrun-style environment variables."""
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    return rank, local, world


def local_device_index() -> int:
    """GPU of this rank: LOCAL_RANK, unless RRL_FORCE_DEVICE pins every rank to one GPU
    (rehearsing the multi-rank path on a one-GPU box, together with RRL_DIST_BACKEND=gloo)."""
    forced = os.environ.get("RRL_FORCE_DEVICE")
    return int(forced) if forced not in (None, "") else dist_env()[1]


def collective_timeout() -> datetime.timedelta:
    """The bound on every collective / P2P wait (RRL_COLLECTIVE_TIMEOUT_S, default 600 s).
    Subgroups must be given it explicitly: ``dist.new_group`` does not inherit the default
    group's timeout."""
    return datetime.timedelta(seconds=float(os.environ.get("RRL_COLLECTIVE_TIMEOUT_S", "600")))


def force_collectives() -> bool:
    """RRL_FORCE_COLLECTIVES=1: a one-rank group takes the world > 1 code path."""
    return os.environ.get("RRL_FORCE_COLLECTIVES", "0") == "1"


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def init_distributed(backend: Optional[str] = None, timeout_s: Optional[float] = None) -> "Comm":
    """Initialise the default process group from the environment (torchrun) if world > 1.
    Backend: ``nccl`` (= RCCL over xGMI on ROCm) with GPUs, ``gloo`` on CPU; override with
    RRL_DIST_BACKEND."""
    rank, local, world = dist_env()
    local = local_device_index()
    forced = world == 1 and force_collectives()
    if timeout_s is None:
        # a stalled rank turns into a collective timeout -> the rank exits -> torchrun restarts
        # the group (--max-restarts) and ranks auto-resume from their checkpoints
        timeout_s = float(os.environ.get("RRL_COLLECTIVE_TIMEOUT_S", "600"))
    if (world > 1 or forced) and not dist.is_initialized():
        backend = backend or os.environ.get("RRL_DIST_BACKEND") or None
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if forced and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend == "nccl":
            torch.cuda.set_device(local)
        tmo = datetime.timedelta(seconds=timeout_s)
        restart = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
        if restart > 0:
            # after a torchrun group restart the rendezvous store still holds the dead
            # group's keys (peer addresses); namespace this attempt's keys
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, False,
                                 timeout=tmo)
            store = dist.PrefixStore(f"rrl_attempt_{restart}", base)
            dist.init_process_group(backend=backend, store=store, rank=rank, world_size=world, timeout=tmo)
        else:
            dist.init_process_group(backend=backend, rank=rank, world_size=world, timeout=tmo)
    return Comm()


class Comm:
    """Thin wrapper so single-process code paths need no branches."""

    def __init__(self, group=None, collectives: Optional[bool] = None):
        self.group = group
        self.enabled = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if self.enabled else 1
        self.rank = dist.get_rank(group) if self.enabled else 0
        self.backend = dist.get_backend(group) if self.enabled else "none"
        if collectives is None:
            collectives = force_collectives()
        # ``multi``: the world > 1 code path (real collectives), also for a forced one-rank group
        self.forced = bool(self.enabled and self.world == 1 and collectives)
        self.multi = self.world > 1 or self.forced
        # muted(): collectives become no-ops (same launches otherwise) -- for rank-local eager
        # warm-ups before a graph capture, which other ranks may not run at the same time
        self._muted = False
        # optional utils.tracing.PhaseTimer: every gradient / statistics all-reduce is timed as
        # the "AllReduce" phase (HIP events on the current stream bracket the RCCL call, which
        # the stream waits on); skipped while a hipGraph is being captured
        self.timer = None

    def muted(self):
        """Context manager: this comm's collectives do nothing inside it.  A graph capture is
        preceded by one eager warm-up of the same body; the capture decision is rank-local
        (a new input-buffer set on one rank, agent rows folded on rank 0 only, a per-rank
        cache eviction), so a warm-up that issued real collectives would pair with another
        rank's unrelated calls.  The captured body itself issues no collective until replay,
        and every rank's graphs carry the same collective sequence (one gradient all-reduce
        of P floats per optimiser step), whatever their batch shapes."""
        import contextlib

        @contextlib.contextmanager
        def cm():
            prev, self._muted = self._muted, True
            try:
                yield self
            finally:
                self._muted = prev

        return cm()

    @property
    def is_master(self) -> bool:
        return self.rank == 0

    @property
    def graph_safe(self) -> bool:
        """Collectives of this comm can be captured into a hipGraph: none are issued, or they
        go through RCCL on the device (gloo collectives are host calls)."""
        return (not self.multi) or self.backend == "nccl"

    def all_reduce_sum_(self, t: torch.Tensor) -> torch.Tensor:
        if self.multi and not self._muted:
            tm = self.timer
            if tm is not None and tm.enabled and not (t.is_cuda and torch.cuda.is_current_stream_capturing()):
                with tm.phase("AllReduce"):
                    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    def all_reduce_max_(self, t: torch.Tensor) -> torch.Tensor:
        if self.multi and not self._muted:
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return t

    def all_reduce_min_(self, t: torch.Tensor) -> torch.Tensor:
        if self.multi and not self._muted:
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.group)
        return t

    def broadcast_(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self.multi and not self._muted:
            dist.broadcast(t, src=src, group=self.group)
        return t

    def barrier(self):
        if self.multi:
            if self.backend == "nccl" and torch.cuda.is_available():
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def gather_to(self, t: torch.Tensor, dst: int, out: Optional[List[torch.Tensor]] = None):
        """Rollout fan-in: every rank's ``t`` lands in ``out[rank]`` on ``dst``.

        Implemented as grouped point-to-point send/recv (each actor->learner transfer
        rides its own xGMI link) rather than a ring gather.
        """
        if not self.multi:
            if out is not None:
                out[0].copy_(t)
            return out
        ops = []
        if self.rank == dst:
            assert out is not None and len(out) == self.world
            for r in range(self.world):
                if r == dst:
                    out[r].copy_(t)
                else:
                    ops.append(dist.P2POp(dist.irecv, out[r], r, self.group))
        else:
            ops.append(dist.P2POp(dist.isend, t, dst, self.group))
        if ops:
            if t.is_cuda and self.backend != "nccl":
                # gloo moves device bytes from host threads, outside stream order (RCCL P2P is
                # stream-ordered): the kernels writing ``t`` / still reading ``out`` must be done
                torch.cuda.current_stream(t.device).synchronize()
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return out

    def all_gather_object(self, obj):
        if not self.multi:
            return [obj]
        res = [None] * self.world
        dist.all_gather_object(res, obj, group=self.group)
        return res
