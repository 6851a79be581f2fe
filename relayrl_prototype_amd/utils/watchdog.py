"""Per-step stall watchdog for the multi-rank engines (SURVEY §5.3 failure detection).

A rank whose peer stops sending (a hung or dead actor, a stuck learner shard) blocks in a
collective or a point-to-point receive until the process-group timeout -- 10 minutes by
default, far longer than an epoch.  ``StepWatchdog`` bounds every step by a budget derived
from the measured step time (``factor`` x its running average, never below
``min_timeout_s``).  When a step overruns, ``diagnose()`` names what the rank is waiting on
(the actors whose rollout has not arrived, with their last heartbeat sequence numbers), the
message is reported, and the process exits with ``EXIT_STALL``: torchrun (--max-restarts)
then restarts the whole group and every rank resumes from its own checkpoint
(runtime/launcher.py --auto-resume).  The reference had no failure detection beyond
per-request retries (agent_grpc.rs:528-531, agent_zmq.rs:662-667).
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Callable, Optional

EXIT_STALL = 75


class StepWatchdog:
    def __init__(self, name: str, min_timeout_s: float = 120.0, factor: float = 20.0,
                 diagnose: Optional[Callable[[], str]] = None, on_stall: Optional[Callable[[str], None]] = None,
                 exit_fn: Callable[[int], None] = os._exit, poll_s: float = 0.1):
        self.name = name
        self.min_timeout_s = float(min_timeout_s)
        self.factor = float(factor)
        self.diagnose = diagnose
        self.on_stall = on_stall
        self.exit_fn = exit_fn
        self.poll_s = poll_s
        self.enabled = self.min_timeout_s > 0
        self._lock = threading.Lock()
        self._t0: Optional[float] = None
        self._step = 0
        self._avg: Optional[float] = None
        self._stop = threading.Event()
        self.fired = False
        self._thread: Optional[threading.Thread] = None
        if self.enabled:
            self._thread = threading.Thread(target=self._run, name=f"rrl-watchdog-{name}", daemon=True)
            self._thread.start()

    def budget(self) -> float:
        avg = self._avg
        return self.min_timeout_s if avg is None else max(self.min_timeout_s, self.factor * avg)

    def begin(self, step: int):
        with self._lock:
            self._t0 = time.monotonic()
            self._step = step

    def end(self):
        with self._lock:
            if self._t0 is None:
                return
            dt = time.monotonic() - self._t0
            self._avg = dt if self._avg is None else 0.9 * self._avg + 0.1 * dt
            self._t0 = None

    def _run(self):
        while not self._stop.wait(self.poll_s):
            with self._lock:
                t0, step = self._t0, self._step
            if t0 is None:
                continue
            el = time.monotonic() - t0
            b = self.budget()
            if el <= b:
                continue
            why = ""
            try:
                why = self.diagnose() if self.diagnose else ""
            except Exception as e:  # the diagnosis must never keep the rank alive
                why = f"(diagnosis failed: {e!r})"
            msg = f"[watchdog] {self.name}: step {step} stalled for {el:.1f} s (budget {b:.1f} s); {why}"
            self.fired = True
            try:
                print(msg, file=sys.stderr, flush=True)
                if self.on_stall:
                    self.on_stall(msg)
            finally:
                self.exit_fn(EXIT_STALL)
            return

    def close(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=1.0)
