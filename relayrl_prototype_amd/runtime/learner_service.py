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
    """``algorithm`` is a built-in (flat-weight ``get_weights()``) or any ``AlgorithmAbstract``
    plugin (rf/README.md:156-229): a plugin's model is the TorchScript file its ``save()`` writes
    (``save_model_path`` attribute, else ``model_path`` = the config's server model path), read
    back after every update and published as a TorchScript-payload blob -- what the reference
    server does (training_zmq.rs:752-785, 901-919: save_model, then the file's bytes to agents).
    Plugins receive every upload in the reference's per-action layout (``as_reference_trajectory``)."""

    def __init__(self, algorithm, max_queue: int = 100000, checkpoint_fn=None, model_path: Optional[str] = None):
        self.algorithm = algorithm
        self.model_path = model_path
        self.plugin = not callable(getattr(algorithm, "get_weights", None))
        self._plugin_version = 0
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
        """Publish the algorithm's current model.  Returns after a pointer swap: transports
        deliver on their own threads (model_store.LatestWorker); the TorchScript archive of a
        built-in is built from the blob's own weights, lazily, by whoever needs it."""
        if self.plugin:
            blob = self._plugin_blob()
        else:
            w = self.algorithm.get_weights()
            meta = {k: w[k] for k in ("obs_dim", "act_dim", "hidden", "discrete")}
            meta["algorithm"] = type(self.algorithm).__name__
            blob = ModelBlob(int(w["version"]), meta, w["pi"].numpy(),
                             None if w.get("vf") is None else w["vf"].numpy())
        self.store.publish(blob)
        return blob

    def _plugin_model_file(self) -> str:
        p = getattr(self.algorithm, "save_model_path", None) or self.model_path
        if not p:
            raise RuntimeError(f"plugin {type(self.algorithm).__name__} has no save_model_path and the server no "
                               "model path: cannot locate the TorchScript its save() writes")
        return str(p)

    def _plugin_blob(self) -> ModelBlob:
        self.algorithm.save()
        with open(self._plugin_model_file(), "rb") as f:
            archive = f.read()
        self._plugin_version += 1
        return ModelBlob.from_torchscript(self._plugin_version, archive, {"algorithm": type(self.algorithm).__name__})

    # ------------------------------------------------------------------ agents
    def register_agent(self, agent_id: str, info: Optional[Dict[str, Any]] = None):
        with self._agents_lock:
            rec = self.agents.setdefault(agent_id, {"seq": -1, "last_seen": time.time(), "trajectories": 0})
            rec.update(info or {})
            rec["last_seen"] = time.time()

    def forget_agents(self, agent_ids) -> None:
        """A transport found these agents unreachable (e.g. a reference PULL gone): stop
        tracking them; one that comes back re-registers through its handshake."""
        with self._agents_lock:
            for a in agent_ids:
                if a in self.agents:
                    self.evicted[a] = self.agents.pop(a)

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
        if self.plugin:
            from ..types import as_reference_trajectory

            traj = as_reference_trajectory(traj)
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
