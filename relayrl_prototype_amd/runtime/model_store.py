"""Versioned model blobs published by the learner to actors / agents.

The reference shipped a TorchScript archive through the filesystem for every update
(server_model.pt -> bytes -> client_model.pt -> CModule::load) and never
versioned it (gRPC version always 0, A5).  Here the learner publishes an immutable
``ModelBlob`` = (monotonic version, flat fp32 policy / value vectors, shape metadata);
transports ship it as an ``RRLM`` frame (a few hundred KB, no file I/O), and the
TorchScript archive is produced lazily only for clients that ask for it (compat).

Custom algorithm plugins (rf/README.md:156-229) own an arbitrary TorchScript model instead of
flat MLP weights: their blob carries the archive the plugin's ``save()`` wrote
(``meta["payload"] == "torchscript"``, see ``ModelBlob.from_torchscript``) and agents run its
``step`` (models/ts_policy.py).

Delivery never runs on the publisher's thread: ``ModelStore.publish`` only swaps the latest
cell and wakes subscribers; transports subscribe through ``LatestWorker``, a thread per
subscriber that always sends the NEWEST blob (an agent that is slow or gone delays only its
own worker, never the learner -- the reference's libzmq PUSH queued and returned the same way,
training_zmq.rs:876-934).
"""
from __future__ import annotations

import json
import struct
import threading
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

import numpy as np

_MAGIC = b"RRLM"


@dataclass
class ModelBlob:
    version: int
    meta: Dict[str, Any]
    pi: np.ndarray
    vf: Optional[np.ndarray] = None
    _ts: Optional[bytes] = field(default=None, repr=False)
    _ts_fn: Optional[Callable[[], bytes]] = field(default=None, repr=False)

    @staticmethod
    def from_torchscript(version: int, archive: bytes, meta: Optional[Dict[str, Any]] = None) -> "ModelBlob":
        """A plugin's model: the TorchScript archive itself is the payload (no flat weights)."""
        m = dict(meta or {})
        m["payload"] = "torchscript"
        return ModelBlob(int(version), m, np.zeros(0, np.float32), None, _ts=bytes(archive))

    @property
    def is_torchscript(self) -> bool:
        return self.meta.get("payload") == "torchscript"

    def encode(self) -> bytes:
        meta = dict(self.meta)
        meta["version"] = int(self.version)
        mj = json.dumps(meta).encode()
        if self.is_torchscript:  # the archive rides in the first payload section
            pi = self.torchscript()
        else:
            pi = np.ascontiguousarray(self.pi, np.float32).tobytes()
        vf = b"" if self.vf is None else np.ascontiguousarray(self.vf, np.float32).tobytes()
        return _MAGIC + struct.pack("<IQQQ", len(mj), len(pi), len(vf), int(self.version)) + mj + pi + vf

    @staticmethod
    def decode(buf: bytes) -> "ModelBlob":
        if buf[:4] != _MAGIC:
            raise ValueError("not an RRLM model frame")
        hdr = struct.calcsize("<IQQQ")
        lm, lp, lv, ver = struct.unpack("<IQQQ", buf[4:4 + hdr])
        o = 4 + hdr
        if o + lm + lp + lv != len(buf):
            raise ValueError("RRLM frame size mismatch")
        meta = json.loads(buf[o:o + lm].decode())
        o += lm
        if meta.get("payload") == "torchscript":
            return ModelBlob.from_torchscript(ver, bytes(buf[o:o + lp]), meta)
        pi = np.frombuffer(buf[o:o + lp], np.float32).copy()
        o += lp
        vf = np.frombuffer(buf[o:o + lv], np.float32).copy() if lv else None
        return ModelBlob(int(ver), meta, pi, vf)

    def torchscript(self) -> bytes:
        """The TorchScript archive of THIS version (built from the blob's own weights, so any
        thread may call it after the learner has moved on; cached)."""
        if self._ts is None:
            if self._ts_fn is not None:
                self._ts = self._ts_fn()
            else:
                from ..models.policies import torchscript_bytes_flat

                self._ts = torchscript_bytes_flat(self.meta["obs_dim"], self.meta["act_dim"], self.meta["hidden"],
                                                  self.pi, self.vf, self.meta.get("discrete", True))
        return self._ts


def blob_from_archive(version: int, archive: bytes) -> ModelBlob:
    """A TorchScript archive received on the reference wire: the built-in MLP layout becomes a
    flat-weight blob (read from the zip's raw storages, nothing executed: the native C++ policy
    runs it); any other architecture stays a TorchScript-payload blob that the agent validates
    and runs through ``step`` (models/ts_policy.py, agent_wrapper.rs:88-168)."""
    from ..utils.checkpoint import reference_weights_from_bytes

    try:
        w = reference_weights_from_bytes(archive)
    except Exception:  # noqa: BLE001 -- not the MLP layout: a plugin's own network
        return ModelBlob.from_torchscript(version, archive)
    return ModelBlob(int(version), {"obs_dim": w["obs_dim"], "act_dim": w["act_dim"], "hidden": w["hidden"],
                                    "discrete": True}, w["pi"], w["vf"])


class ModelStore:
    """Thread-safe latest-model cell with wait-for-newer (long-poll) support."""

    def __init__(self):
        self._cv = threading.Condition()
        self._blob: Optional[ModelBlob] = None
        self._subs: List[Callable[[ModelBlob], None]] = []

    def publish(self, blob: ModelBlob):
        """O(subscribers) pointer swaps: subscribers must not block (use ``LatestWorker``)."""
        with self._cv:
            self._blob = blob
            subs = list(self._subs)
            self._cv.notify_all()
        for s in subs:
            try:
                s(blob)
            except Exception as e:  # a failing subscriber must not break the learner
                print(f"[ModelStore] subscriber error: {e!r}", flush=True)

    def latest(self) -> Optional[ModelBlob]:
        with self._cv:
            return self._blob

    def wait_newer(self, version: int, timeout_s: float) -> Optional[ModelBlob]:
        with self._cv:
            self._cv.wait_for(lambda: self._blob is not None and self._blob.version > version, timeout=timeout_s)
            b = self._blob
            return b if (b is not None and b.version > version) else None

    def subscribe(self, fn: Callable[[ModelBlob], None]):
        with self._cv:
            self._subs.append(fn)

    def unsubscribe(self, fn):
        with self._cv:
            if fn in self._subs:
                self._subs.remove(fn)


class LatestWorker:
    """Runs ``fn(blob)`` on its own thread for the newest published blob only.

    ``ModelStore.subscribe(LatestWorker(fn))``: the publisher's call stores the blob and
    returns; versions published while ``fn`` is still busy collapse into the newest one
    (newest-wins, like a conflating PUB socket).  ``delivered`` / ``skipped`` count versions.
    """

    def __init__(self, fn: Callable[[ModelBlob], None], name: str = "rrl-model-publisher"):
        self.fn = fn
        self._cv = threading.Condition()
        self._pending: Optional[ModelBlob] = None
        self._stop = False
        self.delivered = 0
        self.skipped = 0
        self.errors = 0
        self._busy = False
        self._thread = threading.Thread(target=self._run, name=name, daemon=True)
        self._thread.start()

    def __call__(self, blob: ModelBlob) -> None:
        with self._cv:
            if self._pending is not None:
                self.skipped += 1
            self._pending = blob
            self._cv.notify()

    def _run(self):
        while True:
            with self._cv:
                self._cv.wait_for(lambda: self._stop or self._pending is not None)
                if self._stop:
                    return
                blob, self._pending = self._pending, None
                self._busy = True
            try:
                self.fn(blob)
                self.delivered += 1
            except Exception as e:  # a failing transport must not kill the publisher
                self.errors += 1
                print(f"[LatestWorker] delivery failed: {e!r}", flush=True)
            finally:
                with self._cv:
                    self._busy = False
                    self._cv.notify_all()

    def flush(self, timeout_s: float = 10.0) -> bool:
        """Wait until every published blob has been handed to ``fn`` (tests / shutdown)."""
        with self._cv:
            return self._cv.wait_for(lambda: self._pending is None and not self._busy, timeout=timeout_s)

    def close(self, timeout_s: float = 5.0) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._thread.join(timeout=timeout_s)
