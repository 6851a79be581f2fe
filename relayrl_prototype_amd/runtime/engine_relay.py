"""In-memory link between a TrainingServer (API process) and rank 0 of its multi-GPU engine.

With ``world_size > 1`` the engine's ranks run in a ``torch.distributed.run`` child (one rank
per GPU, RCCL between them).  The API process keeps the agent endpoints (ZMQ / gRPC / local,
bound at construction like the reference's TrainingServer) and this relay closes the
reference's defining loop across the process boundary:

  uploads   agents -> API endpoint -> LearnerService -> RemoteEngineAlgorithm.receive_trajectory
            -> ``TRAJ`` frame (RRLC / RRLT bytes) over a local ZMTP PUSH -> rank 0's PULL ->
            EngineAlgorithm staging -> folded into rank 0's shard of the next epoch
            (training_zmq.rs:948-1058 -> REINFORCE.py:70-95)
  models    rank 0, every ``publish_every`` epochs -> ``MODEL`` frame (RRLM flat weights, from
            rank 0's memory) over a local ZMTP PUSH -> the API process's PULL -> ModelStore ->
            every attached agent (training_zmq.rs:876-934 -> agent_zmq.rs:625-698)
  control   ``STOP`` (background training stopped) API -> rank 0; the ranks agree on it with
            one all-reduce per epoch (EngineRunner.agree_stop)

Nothing on the weight path touches a file (files are checkpoint-only).  Both
links are 127.0.0.1 TCP through the C++ ZMTP sockets (csrc/host/zmtp.cpp): connect is
asynchronous with reconnect, so either side may start first; uploads made before the ranks are
up wait in a bounded queue.
"""
from __future__ import annotations

import queue
import threading
from typing import Callable, Optional

from .. import _native
from ..runtime.model_store import ModelBlob
from ..types import RelayRLTrajectory, TrajectoryColumns

TRAJ = b"TRAJ"
MODEL = b"MODEL"
STOP = b"STOP"


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def encode_upload(traj) -> bytes:
    """An upload as one frame: columnar RRLC, or per-action RRLT (incl. reference frames
    already decoded to actions, terminal markers kept)."""
    if isinstance(traj, TrajectoryColumns):
        return traj.encode()
    return traj.encode()


def decode_upload(buf: bytes):
    if TrajectoryColumns.is_frame(buf):
        return TrajectoryColumns.decode(buf)
    return RelayRLTrajectory.decode(buf)


class ApiRelay:
    """API-process side: PUSH uploads / control to rank 0, PULL models from rank 0."""

    def __init__(self, max_backlog: int = 65536):
        self.down = _native.ZmtpSocket(_native.SockType.PULL)
        self.down_port = self.down.bind("tcp://127.0.0.1:0")
        self.up_port = _free_port()  # rank 0 binds its PULL here
        self.up = _native.ZmtpSocket(_native.SockType.PUSH)
        self.up.connect(f"tcp://127.0.0.1:{self.up_port}")
        self._q: "queue.Queue" = queue.Queue(maxsize=max_backlog)
        self._stop = threading.Event()
        self.forwarded = 0
        self.dropped = 0
        self.models = 0
        self._on_model: Optional[Callable[[ModelBlob], None]] = None
        self._threads = [threading.Thread(target=self._send_loop, daemon=True, name="rrl-relay-up"),
                         threading.Thread(target=self._recv_loop, daemon=True, name="rrl-relay-down")]
        for t in self._threads:
            t.start()

    def argv(self):
        return ["--relay-up", str(self.up_port), "--relay-down", str(self.down_port)]

    def on_model(self, fn: Callable[[ModelBlob], None]) -> None:
        self._on_model = fn

    def send_upload(self, traj) -> bool:
        try:
            self._q.put_nowait([TRAJ, encode_upload(traj)])
            return True
        except queue.Full:
            self.dropped += 1
            return False

    def send_stop(self) -> None:
        self._q.put([STOP])

    def _send_loop(self):
        while not self._stop.is_set():
            try:
                frames = self._q.get(timeout=0.1)
            except queue.Empty:
                continue
            # blocks until rank 0's PULL is up (the ranks may still be starting)
            while not self._stop.is_set():
                if self.up.send(frames, 200):
                    if frames[0] == TRAJ:
                        self.forwarded += 1
                    break

    def _recv_loop(self):
        while not self._stop.is_set():
            msg = self.down.recv(100)
            if msg is None:
                continue
            frames = msg[1]
            if len(frames) >= 2 and frames[0] == MODEL:
                try:
                    blob = ModelBlob.decode(frames[1])
                except ValueError:
                    continue
                self.models += 1
                if self._on_model is not None:
                    self._on_model(blob)

    def close(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self.up.close()
        self.down.close()


class RankRelay:
    """Rank-0 side: PULL uploads / control from the API process, PUSH models to it."""

    def __init__(self, up_port: int, down_port: int, on_upload: Callable, on_stop: Callable[[], None]):
        self.pull = _native.ZmtpSocket(_native.SockType.PULL)
        self.pull.bind(f"tcp://127.0.0.1:{int(up_port)}")
        self.push = _native.ZmtpSocket(_native.SockType.PUSH)
        self.push.connect(f"tcp://127.0.0.1:{int(down_port)}")
        self.on_upload = on_upload
        self.on_stop = on_stop
        self.received = 0
        self.bad = 0
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._loop, daemon=True, name="rrl-rank-relay")
        self._t.start()

    def _loop(self):
        while not self._stop.is_set():
            msg = self.pull.recv(100)
            if msg is None:
                continue
            frames = msg[1]
            if not frames:
                continue
            if frames[0] == STOP:
                self.on_stop()
            elif frames[0] == TRAJ and len(frames) >= 2:
                try:
                    traj = decode_upload(frames[1])
                except Exception:  # noqa: BLE001 -- a bad frame must not end the rank
                    self.bad += 1
                    continue
                self.received += 1
                self.on_upload(traj)

    def send_model(self, blob: ModelBlob, timeout_ms: int = 2000) -> bool:
        return bool(self.push.send([MODEL, blob.encode()], timeout_ms))

    def close(self):
        self._stop.set()
        self._t.join(timeout=5)
        self.pull.close()
        self.push.close()
