"""In-process learner service: the replacement for the reference's Python learner
subprocess + stdin/stdout JSON bridge (python_algorithm_request.rs, python_algorithm_reply.py;
SURVEY §2.7 C6 "eliminated").

Transports call ``submit(trajectory)``; a single worker thread feeds the algorithm in
arrival order (the reference serialised the same way with one lock), publishes a new
``ModelBlob`` whenever the algorithm reports an update, and tracks per-agent
heartbeats (last sequence number / time) for failure detection.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Any, Dict, Optional

from .model_store import ModelBlob, ModelStore


class LearnerService:
    def __init__(self, algorithm, max_queue: int = 100000, checkpoint_fn=None):
        self.algorithm = algorithm
        self.store = ModelStore()
        self.q: "queue.Queue" = queue.Queue(maxsize=max_queue)
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.agents: Dict[str, Dict[str, Any]] = {}
        self._agents_lock = threading.Lock()
        self.received = 0
        self.updates = 0
        self.dropped_seq = 0
        self.errors = 0
        self.last_error: Optional[str] = None
        self.checkpoint_fn = checkpoint_fn
        self.evicted: Dict[str, Dict[str, Any]] = {}
        self._evict_cbs = []
        self._sweeper: Optional[threading.Thread] = None
        self._stop_sweep = threading.Event()
        self.publish_model()

    # ------------------------------------------------------------------ models
    def publish_model(self) -> ModelBlob:
        w = self.algorithm.get_weights()
        meta = {k: w[k] for k in ("obs_dim", "act_dim", "hidden", "discrete")}
        meta["algorithm"] = type(self.algorithm).__name__
        blob = ModelBlob(int(w["version"]), meta, w["pi"].numpy(), None if w.get("vf") is None else w["vf"].numpy(),
                         _ts_fn=self.algorithm.model_bytes)
        self.store.publish(blob)
        return blob

    # ------------------------------------------------------------------ agents
    def register_agent(self, agent_id: str, info: Optional[Dict[str, Any]] = None):
        with self._agents_lock:
            rec = self.agents.setdefault(agent_id, {"seq": -1, "last_seen": time.time(), "trajectories": 0})
            rec.update(info or {})
            rec["last_seen"] = time.time()

    def stale_agents(self, timeout_s: float):
        now = time.time()
        with self._agents_lock:
            return [a for a, r in self.agents.items() if now - r["last_seen"] > timeout_s]

    def on_evict(self, fn) -> None:
        """``fn(agent_ids)`` runs after each eviction (transports drop their routing state)."""
        self._evict_cbs.append(fn)

    def evict_stale(self, timeout_s: float) -> list:
        """Drop agents silent for ``timeout_s`` (no upload, heartbeat or handshake): they stop
        receiving model pushes; an evicted agent that comes back simply re-registers."""
        now = time.time()
        with self._agents_lock:
            # ``exempt`` = a peer without any liveness signal (reference agents, zmq_transport.py)
            gone = [a for a, r in self.agents.items() if now - r["last_seen"] > timeout_s and not r.get("exempt")]
            for a in gone:
                self.evicted[a] = self.agents.pop(a)
        if gone:
            print(f"[LearnerService] evicted {len(gone)} silent agent(s) (> {timeout_s:.0f} s): {gone}", flush=True)
            for fn in list(self._evict_cbs):
                try:
                    fn(gone)
                except Exception as e:
                    print(f"[LearnerService] eviction hook failed: {e!r}", flush=True)
        return gone

    def start_sweeper(self, timeout_s: float, period_s: float = 5.0) -> None:
        """Periodic ``evict_stale`` in a daemon thread."""
        if timeout_s <= 0 or (self._sweeper is not None and self._sweeper.is_alive()):
            return

        def loop():
            while not self._stop_sweep.wait(period_s):
                self.evict_stale(timeout_s)

        self._stop_sweep.clear()
        self._sweeper = threading.Thread(target=loop, name="relayrl-agent-sweeper", daemon=True)
        self._sweeper.start()

    def stop_sweeper(self) -> None:
        self._stop_sweep.set()
        if self._sweeper is not None:
            self._sweeper.join(timeout=5)
        self._sweeper = None

    # ------------------------------------------------------------------ ingest
    def submit(self, traj, block: bool = True, timeout: Optional[float] = None) -> bool:
        try:
            self.q.put(traj, block=block, timeout=timeout)
            return True
        except queue.Full:
            return False

    def process(self, traj) -> bool:
        """Synchronous ingest (also used by the worker thread)."""
        aid = getattr(traj, "agent_id", "") or ""
        if aid:
            with self._agents_lock:
                rec = self.agents.setdefault(aid, {"seq": -1, "last_seen": 0.0, "trajectories": 0})
                seq = getattr(traj, "seq", 0)
                if rec["seq"] >= 0 and seq > rec["seq"] + 1:
                    self.dropped_seq += seq - rec["seq"] - 1  # lost uploads (heartbeat gap)
                rec["seq"] = max(rec["seq"], seq)
                rec["last_seen"] = time.time()
                rec["trajectories"] += 1
        self.received += 1
        updated = bool(self.algorithm.receive_trajectory(traj))
        if updated:
            self.updates += 1
            self.publish_model()
            if self.checkpoint_fn is not None:
                self.checkpoint_fn(self)
        return updated

    def _run(self):
        while not self._stop.is_set():
            try:
                traj = self.q.get(timeout=0.05)
            except queue.Empty:
                continue
            try:
                self.process(traj)
            except Exception as e:  # keep serving; surface the error
                self.errors += 1
                self.last_error = repr(e)
                print(f"[LearnerService] error while training: {e!r}", flush=True)
            finally:
                self.q.task_done()

    def start(self):
        if self._thread is None or not self._thread.is_alive():
            self._stop.clear()
            self._thread = threading.Thread(target=self._run, name="relayrl-learner", daemon=True)
            self._thread.start()

    def stop(self, drain: bool = False, timeout: float = 30.0):
        if drain:
            t0 = time.time()
            while not self.q.empty() and time.time() - t0 < timeout:
                time.sleep(0.01)
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=timeout)
        self._thread = None

    def join_queue(self, timeout: float = 60.0) -> bool:
        t0 = time.time()
        while time.time() - t0 < timeout:
            if self.q.unfinished_tasks == 0:
                return True
            time.sleep(0.005)
        return False
