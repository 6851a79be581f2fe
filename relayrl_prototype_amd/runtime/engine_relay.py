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
  control   ``HELLO <port>`` rank 0 -> API: rank 0 binds its upload PULL on a free port (no
            port picked, closed and re-bound across processes) and reports it; the API
            process then connects its upload PUSH.  ``STOP`` (background training stopped)
            API -> rank 0, sent ahead of any queued upload; the ranks agree on it through the
            per-epoch all-reduce the engine already runs (EngineRunner.agree_stop)

Nothing on the weight path touches a file (files are checkpoint-only).  Both
links are 127.0.0.1 TCP through the C++ ZMTP sockets (csrc/host/zmtp.cpp): connect is
asynchronous with reconnect, so either side may start first; uploads made before the ranks are
up wait in a bounded queue.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Callable, Optional

from .. import _native
from ..runtime.model_store import ModelBlob
from ..types import RelayRLTrajectory, TrajectoryColumns

TRAJ = b"TRAJ"
MODEL = b"MODEL"
STOP = b"STOP"
HELLO = b"HELLO"


def encode_upload(traj) -> bytes:
    """An upload as one frame: columnar RRLC (TrajectoryColumns), or per-action RRLT
    (RelayRLTrajectory, incl. reference frames already decoded to actions, terminal markers
    kept) -- both types encode themselves."""
    return traj.encode()


def decode_upload(buf: bytes):
    if TrajectoryColumns.is_frame(buf):
        return TrajectoryColumns.decode(buf)
    return RelayRLTrajectory.decode(buf)


class ApiRelay:
    """API-process side: PUSH uploads / control to rank 0, PULL models (and rank 0's HELLO)."""

    def __init__(self, max_backlog: int = 65536):
        self.down = _native.ZmtpSocket(_native.SockType.PULL)
        self.down_port = self.down.bind("tcp://127.0.0.1:0")
        self.up = None  # connected when rank 0 reports its upload port (HELLO)
        self.up_port = None
        self._up_lock = threading.Lock()
        self._q: "queue.Queue" = queue.Queue(maxsize=max_backlog)
        self._stop = threading.Event()
        self._stop_req = threading.Event()  # a STOP to deliver ahead of the queued uploads
        self.forwarded = 0
        self.dropped = 0
        self.models = 0
        self._on_model: Optional[Callable[[ModelBlob], None]] = None
        self._threads = [threading.Thread(target=self._send_loop, daemon=True, name="rrl-relay-up"),
                         threading.Thread(target=self._recv_loop, daemon=True, name="rrl-relay-down")]
        for t in self._threads:
            t.start()

    def argv(self):
        return ["--relay-up", "0", "--relay-down", str(self.down_port)]

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
        """Never blocks: a flag the send loop serves before any queued upload."""
        self._stop_req.set()

    def reset_control(self) -> None:
        """Before a new train(): a STOP meant for the previous run must not end this one, and
        the previous ranks' upload port is gone."""
        self._stop_req.clear()
        with self._up_lock:
            if self.up is not None:
                self.up.close()
            self.up, self.up_port = None, None

    def _connect_up(self, port: int) -> None:
        with self._up_lock:
            if self.up_port == port:
                return
            if self.up is not None:
                self.up.close()
            self.up = _native.ZmtpSocket(_native.SockType.PUSH)
            self.up.connect(f"tcp://127.0.0.1:{port}")
            self.up_port = port

    def _send(self, frames) -> bool:
        with self._up_lock:
            up = self.up
        return up is not None and up.send(frames, 200)

    def _send_loop(self):
        pending = None
        while not self._stop.is_set():
            if self._stop_req.is_set():
                if self._send([STOP]):
                    self._stop_req.clear()
                else:
                    time.sleep(0.01)  # rank 0 not up (yet / any more)
                continue
            if pending is None:
                try:
                    pending = self._q.get(timeout=0.05)
                except queue.Empty:
                    continue
            # waits (in 200 ms slices, STOP first) until rank 0's PULL is up
            if self._send(pending):
                self.forwarded += 1
                pending = None
            elif self.up is None:
                time.sleep(0.01)

    def _recv_loop(self):
        while not self._stop.is_set():
            msg = self.down.recv(100)
            if msg is None:
                continue
            frames = msg[1]
            if len(frames) >= 2 and frames[0] == HELLO:
                try:
                    self._connect_up(int(bytes(frames[1]).decode()))
                except ValueError:
                    continue
            elif len(frames) >= 2 and frames[0] == MODEL:
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
        with self._up_lock:
            if self.up is not None:
                self.up.close()
        self.down.close()


class RankRelay:
    """Rank-0 side: PULL uploads / control from the API process, PUSH models to it."""

    def __init__(self, up_port: int, down_port: int, on_upload: Callable, on_stop: Callable[[], None]):
        """``up_port`` 0: bind a free port and report it to the API process (HELLO)."""
        self.pull = _native.ZmtpSocket(_native.SockType.PULL)
        self.port = self.pull.bind(f"tcp://127.0.0.1:{int(up_port or 0)}")
        self.push = _native.ZmtpSocket(_native.SockType.PUSH)
        self.push.connect(f"tcp://127.0.0.1:{int(down_port)}")
        if not self.push.send([HELLO, str(self.port).encode()], 30000):
            raise RuntimeError("engine relay: the API process did not accept rank 0's HELLO")
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
