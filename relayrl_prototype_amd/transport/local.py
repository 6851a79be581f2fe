"""In-process transport (server_type="local"): agent and learner share the process, so a
trajectory is handed over by reference and model updates are a pointer swap.  This is
the minimum end-to-end slice of SURVEY §7.3 and the fastest path for single-process use.
"""
from __future__ import annotations

import threading
from typing import Dict

_REG: Dict[str, object] = {}
_LOCK = threading.Lock()


def register(address: str, service) -> None:
    with _LOCK:
        _REG[address] = service


def unregister(address: str, service=None) -> None:
    with _LOCK:
        if address in _REG and (service is None or _REG[address] is service):
            del _REG[address]


def lookup(address: str):
    with _LOCK:
        s = _REG.get(address)
    if s is None:
        raise ConnectionError(f"no local training server registered at {address!r}")
    return s


class LocalAgentTransport:
    def __init__(self, address: str, on_model, agent_id: str):
        self.service = lookup(address)
        self.on_model = on_model
        self.agent_id = agent_id
        self._worker = None
        self.service.register_agent(agent_id)
        self.service.store.subscribe(self._on_model)
        blob = self.service.store.latest()
        if blob is not None:
            on_model(blob)

    def _on_model(self, blob):
        if blob.is_torchscript:  # a plugin's archive: loaded + validated off the learner thread
            if self._worker is None:
                from ..runtime.model_store import LatestWorker

                self._worker = LatestWorker(self.on_model, name="rrl-local-model")
            self._worker(blob)
        else:  # flat weights: a pointer swap / memcpy into the native policy
            self.on_model(blob)

    def send_trajectory_obj(self, traj) -> bool:
        return self.service.submit(traj)

    def close(self):
        self.service.store.unsubscribe(self._on_model)
        if self._worker is not None:
            self._worker.close()
