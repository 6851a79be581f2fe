"""Elastic shrink: the survivors of a stalled rank re-form the process group without it and
keep training ("the learner detects a stalled rank by timeout and re-forms the
comm without it").

The reference has no failure handling beyond per-request retries and hard exits
(agent_grpc.rs:528-531, agent_zmq.rs:662-667).  Here:

* A long-lived control store (``torch.distributed.TCPStore``) is hosted by rank 0 for the
  whole job.  Every process-group generation ``g`` initialises from it under the key prefix
  ``pg{g}/``, so a new group can be formed after the old one broke.
* A stalled peer turns into an exception in the survivors' next collective or P2P wait:
  the process-group timeout (``RRL_COLLECTIVE_TIMEOUT_S``) bounds every wait, and once one
  survivor has left the group the others' operations fail at once.
* ``reform()``: every survivor marks itself alive under ``alive/{g}/{rank}``.  The leader
  (the lowest surviving original rank) waits up to ``grace_s`` for the members, publishes the
  new member list under ``reform/{g}``, and everyone re-initialises with its new rank.  A
  rank that is not in the list is evicted: ``reform()`` raises ``Evicted`` and a monitor thread
  ends a rank that is still hung inside a collective (exit code 0, so torchrun does not tear
  the survivors down).
* A crashed rank (non-zero exit) is left to torchrun: it restarts the group and the ranks
  auto-resume from their checkpoints (runtime/launcher.py --max-restarts / --auto-resume).
  If the leader itself is gone, the others time out waiting for ``reform/{g}`` and fail the
  same way.
"""
from __future__ import annotations

import datetime
import json
import os
import threading
import time
from typing import List, Optional

import torch.distributed as dist

from .comm import Comm, dist_env


class Evicted(RuntimeError):
    """This rank was dropped from the group by the survivors."""


class ElasticGroup:
    def __init__(self, backend: Optional[str] = None, timeout_s: Optional[float] = None,
                 grace_s: Optional[float] = None, control_port: Optional[int] = None):
        import torch

        rank, _, world = dist_env()
        self.orig_rank = rank
        self.members: List[int] = list(range(world))
        self.initial_world = world
        self.gen = 0
        self.backend = backend or os.environ.get("RRL_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        self.timeout_s = float(timeout_s if timeout_s is not None else os.environ.get("RRL_COLLECTIVE_TIMEOUT_S", "600"))
        # survivors leave the broken group in a cascade (a rank blocked on the lost peer waits
        # out its timeout; the others fail once a survivor has left), so they reach reform()
        # up to a couple of timeouts apart: the leader collects members for 2 timeouts + 5 s,
        # the others wait for its decision longer than that
        self.grace_s = float(grace_s if grace_s is not None else 2 * self.timeout_s + 5.0)
        if self.backend == "nccl":
            # RCCL: on a collective timeout abort the communicator and raise in the caller
            # (CleanUpOnly) instead of the default that ends the process
            os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "2")
        host = os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if control_port is None:
            control_port = int(os.environ.get("RRL_CONTROL_PORT") or int(os.environ.get("MASTER_PORT", "29500")) + 1)
        self.store = dist.TCPStore(host, int(control_port), None, rank == 0,
                                   timeout=datetime.timedelta(seconds=max(60.0, 2 * self.grace_s + 3 * self.timeout_s)),
                                   wait_for_workers=False)
        self.reforms = 0
        self._stop = threading.Event()
        self._mon = threading.Thread(target=self._monitor, name="rrl-elastic-monitor", daemon=True)
        self._mon.start()

    # ------------------------------------------------------------------ groups
    @property
    def rank(self) -> int:
        return self.members.index(self.orig_rank)

    @property
    def world(self) -> int:
        return len(self.members)

    def init_group(self) -> Comm:
        """Initialise process-group generation ``self.gen`` from the control store."""
        if self.backend == "nccl":
            import torch

            from .comm import local_device_index

            torch.cuda.set_device(local_device_index())
        dist.init_process_group(self.backend, store=dist.PrefixStore(f"pg{self.gen}", self.store), rank=self.rank,
                                world_size=self.world, timeout=datetime.timedelta(seconds=self.timeout_s))
        return Comm()

    def reform(self) -> Comm:
        """Called by a survivor whose collective failed: agree on the members still alive,
        drop the others, and return the new generation's Comm (raises Evicted if this rank is
        no longer a member, RuntimeError if no decision arrives)."""
        try:
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
        g = self.gen
        self.store.set(f"alive/{g}/{self.orig_rank}", "1")
        leader = self.members[0]
        if self.orig_rank == leader:
            deadline = time.monotonic() + self.grace_s
            while time.monotonic() < deadline:
                if all(self.store.check([f"alive/{g}/{m}"]) for m in self.members):
                    break
                time.sleep(0.05)
            alive = [m for m in self.members if self.store.check([f"alive/{g}/{m}"])]
            self.store.set(f"reform/{g}", json.dumps(alive))
        else:
            try:
                self.store.wait([f"reform/{g}"], datetime.timedelta(seconds=self.grace_s + 3 * self.timeout_s + 10))
            except Exception as e:  # the leader is gone too: fall back to a group restart
                raise RuntimeError(f"elastic reform {g}: no decision from leader rank {leader}") from e
        members = json.loads(self.store.get(f"reform/{g}"))
        if self.orig_rank not in members:
            self._mark_gone()
            raise Evicted(f"rank {self.orig_rank} evicted at reform {g} (members {members})")
        changed = members != self.members
        self.members = members
        self.gen = g + 1
        self.reforms += 1
        comm = self.init_group()
        if not changed:
            # everyone is alive: the failure was not a lost peer -- let the caller re-raise
            comm.unchanged = True
        return comm

    def evicted(self) -> bool:
        """True once a decision for the current generation excludes this rank."""
        g = self.gen
        if not self.store.check([f"reform/{g}"]):
            return False
        return self.orig_rank not in json.loads(self.store.get(f"reform/{g}"))

    def _mark_gone(self):
        try:
            self.store.set(f"gone/{self.orig_rank}", "1")
        except Exception:
            pass

    def _monitor(self):
        # a rank hung inside a collective cannot run reform(): end it once the survivors have
        # decided without it (exit 0 -- torchrun must not restart the survivors)
        while not self._stop.wait(0.5):
            try:
                if self.evicted():
                    print(f"[elastic] rank {self.orig_rank} evicted at reform {self.gen}; exiting", flush=True)
                    self._mark_gone()
                    os._exit(0)
            except Exception:
                return

    def close(self, wait_evicted_s: float = 15.0):
        """Stop the monitor.  Rank 0 hosts the control store: it waits (bounded) for every
        rank it evicted to have left, so a rank still hung in a collective sees the decision
        before the store goes away with this process."""
        self._stop.set()
        if self.orig_rank != 0:
            return
        gone = [r for r in range(self.initial_world) if r not in self.members]
        deadline = time.monotonic() + wait_evicted_s
        while gone and time.monotonic() < deadline:
            gone = [r for r in gone if not self.store.check([f"gone/{r}"])]
            time.sleep(0.1)
