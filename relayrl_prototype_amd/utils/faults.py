"""Fault injection for transport / runtime robustness tests.

Configured by the ``RRL_FAULTS`` environment variable (or ``FaultInjector.configure``):

    RRL_FAULTS="drop=0.1,corrupt=0.05,delay_ms=20,seed=3"

* ``drop``     -- probability that an outgoing trajectory upload is silently dropped
                  (the learner sees the per-agent sequence gap: LearnerService.dropped_seq);
* ``corrupt``  -- probability that an upload has bytes flipped (the server must reject
                  the frame and keep serving);
* ``delay_ms`` -- fixed delay added before each upload (slow agent).

Off by default; every hook is a no-op unless configured.

Process-level faults for the elastic-restart path (runtime/launcher.py):

    RRL_FAULT_KILL="1:3"   -- rank 1 dies (exit 17) after epoch 3, once per run directory;
                              torchrun (--max-restarts) restarts the group and every rank
                              resumes from its last checkpoint.
    RRL_FAULT_STALL="2:2:60" -- rank 2 hangs for 60 s before epoch 2 (a stuck actor), once
                              per run directory: its peers' step watchdogs
                              (utils/watchdog.py) exit them, torchrun restarts the group.
    RRL_FAULT_STALL_AT="2:3:viter:40:60" -- rank 2 hangs for 60 s at a named site INSIDE
                              epoch 3, once per run directory: ``viter`` = before the 40th
                              value-loop update (its all-reduce), ``gather`` = a learner before
                              receiving its shard, ``send`` = an actor before sending its
                              rollout.  The peers fail mid-epoch, with part of the epoch's
                              updates applied (the elastic epoch-start snapshot's test case).
"""
from __future__ import annotations

import os
import random
import threading
import time
from typing import Dict, Optional


class FaultInjector:
    def __init__(self, spec: Optional[str] = None):
        self._lock = threading.Lock()
        self.configure(spec if spec is not None else os.environ.get("RRL_FAULTS", ""))

    def configure(self, spec: str):
        cfg: Dict[str, float] = {}
        for part in (spec or "").split(","):
            if "=" in part:
                k, v = part.split("=", 1)
                cfg[k.strip()] = float(v)
        self.drop = cfg.get("drop", 0.0)
        self.corrupt = cfg.get("corrupt", 0.0)
        self.delay_ms = cfg.get("delay_ms", 0.0)
        self.rng = random.Random(int(cfg.get("seed", 0)))
        self.enabled = bool(self.drop or self.corrupt or self.delay_ms)
        self.stats = {"dropped": 0, "corrupted": 0, "delayed": 0}

    def filter_upload(self, payload: bytes) -> Optional[bytes]:
        """Returns the (possibly corrupted) payload, or None to drop it."""
        if not self.enabled:
            return payload
        with self._lock:
            if self.delay_ms:
                self.stats["delayed"] += 1
                time.sleep(self.delay_ms / 1000.0)
            if self.drop and self.rng.random() < self.drop:
                self.stats["dropped"] += 1
                return None
            if self.corrupt and self.rng.random() < self.corrupt and len(payload) > 16:
                self.stats["corrupted"] += 1
                b = bytearray(payload)
                for _ in range(4):
                    b[self.rng.randrange(len(b))] ^= 0xFF
                b[0] ^= 0xFF  # always break the magic so decoding must reject it
                return bytes(b)
        return payload


_GLOBAL: Optional[FaultInjector] = None


def injector() -> FaultInjector:
    global _GLOBAL
    if _GLOBAL is None:
        _GLOBAL = FaultInjector()
    return _GLOBAL


def reset(spec: str = "") -> FaultInjector:
    global _GLOBAL
    _GLOBAL = FaultInjector(spec)
    return _GLOBAL


def maybe_kill_rank(rank: int, epoch: int, run_dir: str) -> None:
    """Crash this process once if RRL_FAULT_KILL names (rank, epoch)."""
    spec = os.environ.get("RRL_FAULT_KILL", "")
    if not spec:
        return
    r, e = (int(x) for x in spec.split(":"))
    if r != rank or e != epoch:
        return
    marker = os.path.join(run_dir, f".fault_fired_r{rank}_e{epoch}")
    if os.path.exists(marker):
        return
    os.makedirs(run_dir, exist_ok=True)
    open(marker, "w").close()
    print(f"[faults] injected crash of rank {rank} after epoch {epoch}", flush=True)
    os._exit(17)


def maybe_stall_rank(rank: int, epoch: int, run_dir: str) -> None:
    """Hang this rank once if RRL_FAULT_STALL names (rank, epoch, seconds)."""
    spec = os.environ.get("RRL_FAULT_STALL", "")
    if not spec:
        return
    r, e, sec = spec.split(":")
    if int(r) != rank or int(e) != epoch:
        return
    marker = os.path.join(run_dir, f".stall_fired_r{rank}_e{epoch}")
    if os.path.exists(marker):
        return
    os.makedirs(run_dir, exist_ok=True)
    open(marker, "w").close()
    print(f"[faults] injected stall of rank {rank} before epoch {epoch} ({sec} s)", flush=True)
    time.sleep(float(sec))


_CTX = {"rank": -1, "epoch": -1, "run_dir": "."}
_AT = None  # parsed RRL_FAULT_STALL_AT, or False when unset


def set_context(rank: int, epoch: int, run_dir: str) -> None:
    """The launcher's (original) rank, the epoch about to run and the run directory: the
    coordinates of the mid-epoch stall sites (maybe_stall_at)."""
    _CTX.update(rank=int(rank), epoch=int(epoch), run_dir=run_dir)


def maybe_stall_at(site: str, index: int = 0) -> None:
    """Hang once if RRL_FAULT_STALL_AT names (this rank, the current epoch, ``site``, ``index``)."""
    global _AT
    if _AT is None:
        spec = os.environ.get("RRL_FAULT_STALL_AT", "")
        if spec:
            r, e, st, i, sec = spec.split(":")
            _AT = (int(r), int(e), st, int(i), float(sec))
        else:
            _AT = False
    if not _AT:
        return
    r, e, st, i, sec = _AT
    if (r, e, st, i) != (_CTX["rank"], _CTX["epoch"], site, int(index)):
        return
    marker = os.path.join(_CTX["run_dir"], f".stall_at_fired_r{r}_e{e}_{st}{i}")
    if os.path.exists(marker):
        return
    os.makedirs(_CTX["run_dir"], exist_ok=True)
    open(marker, "w").close()
    print(f"[faults] injected stall of rank {r} in epoch {e} at {st}[{i}] ({sec} s)", flush=True)
    time.sleep(sec)
