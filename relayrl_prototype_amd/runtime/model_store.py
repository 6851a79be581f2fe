"""Versioned model blobs published by the learner to actors / agents.

The reference shipped a TorchScript archive through the filesystem for every update
(server_model.pt -> bytes -> client_model.pt -> CModule::load) and never
versioned it (gRPC version always 0, A5).  Here the learner publishes an immutable
``ModelBlob`` = (monotonic version, flat fp32 policy / value vectors, shape metadata);
transports ship it as an ``RRLM`` frame (a few hundred KB, no file I/O), and the
TorchScript archive is produced lazily only for clients that ask for it (compat).
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

    def encode(self) -> bytes:
        meta = dict(self.meta)
        meta["version"] = int(self.version)
        mj = json.dumps(meta).encode()
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
        pi = np.frombuffer(buf[o:o + lp], np.float32).copy()
        o += lp
        vf = np.frombuffer(buf[o:o + lv], np.float32).copy() if lv else None
        return ModelBlob(int(ver), meta, pi, vf)

    def torchscript(self) -> bytes:
        if self._ts is None:
            if self._ts_fn is not None:
                self._ts = self._ts_fn()
            else:
                from ..models.policies import build_policy_module, torchscript_bytes
                import torch

                m = build_policy_module(self.meta["obs_dim"], self.meta["act_dim"], self.meta["hidden"],
                                        torch.from_numpy(self.pi), None if self.vf is None else torch.from_numpy(self.vf),
                                        self.meta.get("discrete", True))
                self._ts = torchscript_bytes(m)
        return self._ts


class ModelStore:
    """Thread-safe latest-model cell with wait-for-newer (long-poll) support."""

    def __init__(self):
        self._cv = threading.Condition()
        self._blob: Optional[ModelBlob] = None
        self._subs: List[Callable[[ModelBlob], None]] = []

    def publish(self, blob: ModelBlob):
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
