"""ZMTP (ZeroMQ wire protocol) endpoints over the native C++ sockets.

Server side (reference training_zmq.rs:669-1058):
  * ROUTER bound at ``agent_listener``: ``["", "GET_MODEL"(, fmt)]`` -> ``["", model]``;
    ``["", "MODEL_SET"]`` -> register + ``["", "ID_LOGGED"]``; ``["", "HEARTBEAT"]``;
    ``["", "BYE"]``.  Model updates are pushed to every registered agent over the same
    ROUTER socket as ``["", "MODEL", version, blob]`` -- the reference instead connected
    a PUSH to a PULL each agent had to *bind* on one fixed port, which limited it to one
    agent per host (defect A6) and never stopped listening only when multiactor was set.
  * PULL bound at ``trajectory_server``: one frame per episode (fan-in) -- a columnar RRLC
    frame (agent default), a per-action RRLT frame, or a reference agent's
    ``serde_pickle(Vec<RelayRLAction>)`` frame (trajectory.rs:50-90), decoded by the
    data-only opcode interpreter of ``serde_pickle.py`` with the re-sent prefix stripped.
  * Reference agents (GET_MODEL without a format frame, agent_zmq.rs:316-442) get their
    model updates the reference way: a PUSH connected to the ``training_server`` address the
    agent BINDS a PULL on (training_zmq.rs:876-934, agent_zmq.rs:625-698), one TorchScript
    frame per update.
Agent side (agent_zmq.rs:163-698): DEALER (identity = agent id) + PUSH.
No busy polling anywhere (A7): receives block in C++ with timeouts.
"""
from __future__ import annotations

import os
import random
import threading
import time
from typing import Callable, Optional

from .. import _native
from ..runtime.model_store import LatestWorker, ModelBlob
from ..types import ReferenceColumns, RelayRLTrajectory, TrajectoryColumns

FMT_TORCHSCRIPT = b"TORCHSCRIPT"
FMT_RRLM = b"RRLM"


def make_agent_id() -> str:
    """``AGENT_ID-{pid}{rand}`` like agent_zmq.rs:171-174 (plus more entropy)."""
    return f"AGENT_ID-{os.getpid()}{random.randint(0, 99)}-{random.getrandbits(32):08x}"


class ZmqTrainingEndpoint:
    def __init__(self, service, agent_listener: str, trajectory_server: str, multiactor: bool = True,
                 verbose: bool = False, model_push_addr: Optional[str] = None, ref_push_timeout_ms: int = 50,
                 ref_push_max_failures: int = 3, decode_threads: int = 4):
        from .serde_pickle import ReferenceDeduper

        self.service = service
        self.model_push_addr = model_push_addr
        self.ref_agents = set()   # identities that did the reference handshake
        self._model_push = None   # PUSH -> reference agents' bound PULL (lazy)
        self.dedupe = ReferenceDeduper()  # one memory for the column and the per-action decode paths
        from concurrent.futures import ThreadPoolExecutor

        self._decoders = ThreadPoolExecutor(max_workers=decode_threads, thread_name_prefix="rrl-zmq-decode")
        self._last_touch = 0.0
        self.reference_frames = 0
        self.multiactor = multiactor
        self.verbose = verbose
        self.router = _native.ZmtpSocket(_native.SockType.ROUTER)
        self.pull = _native.ZmtpSocket(_native.SockType.PULL)
        self.listener_port = self.router.bind(agent_listener)
        self.traj_port = self.pull.bind(trajectory_server)
        self.agents = {}  # identity -> wants format
        self.bad_frames = 0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._threads = [threading.Thread(target=self._listen_agents, daemon=True, name="rrl-zmq-listener"),
                         threading.Thread(target=self._listen_traj, daemon=True, name="rrl-zmq-traj")]
        for t in self._threads:
            t.start()
        # model delivery runs on its own thread, newest-wins: ModelStore.publish returns at once
        # and a slow or departed agent never stalls the learner (training_zmq.rs:876-934 queued
        # into a libzmq PUSH the same way)
        self.ref_push_timeout_ms = ref_push_timeout_ms
        self.ref_push_max_failures = ref_push_max_failures
        self._ref_push_failures = 0
        self._ref_push_dead = False  # set after N failed pushes; re-armed by GET_MODEL / uploads
        self.ref_pushes = 0
        self.ref_push_timeouts = 0
        self._publisher = LatestWorker(self._on_model, name="rrl-zmq-publisher")
        service.store.subscribe(self._publisher)
        if hasattr(service, "on_evict"):
            service.on_evict(self._on_evict)

    def _on_evict(self, agent_ids):
        """Our agents heartbeat, so silence means gone: drop their push routes.  Reference
        agents have no liveness signal at all (agent_zmq.rs handshakes once at startup and
        never again, and uploads over a fresh PUSH connection each time, so an upload cannot
        be tied to a DEALER identity): they are registered ``exempt`` and never reach this
        hook -- the PUSH to their bound PULL simply times out if one has really gone."""
        ids = {a.encode() if isinstance(a, str) else a for a in agent_ids}
        with self._lock:
            for peer in [p for p in self.agents if p in ids]:
                del self.agents[peer]

    def _rearm_reference_push(self):
        with self._lock:
            self._ref_push_dead = False
            self._ref_push_failures = 0

    def _touch_reference_agents(self):
        """A reference upload arrived: refresh every reference agent's last_seen (the upload's
        PUSH connection carries no identity, training_zmq.rs:971-1012) and re-arm a push route
        dropped after failed sends (the agent is evidently alive)."""
        now = time.monotonic()
        if now - self._last_touch < 0.5:  # liveness has a granularity of seconds: once per 0.5 s
            return
        self._last_touch = now
        self._rearm_reference_push()
        with self._lock:
            ref = list(self.ref_agents)
        for peer in ref:
            self.service.register_agent(peer.decode(errors="replace"))

    def _log(self, *a):
        if self.verbose:
            print("[ZmqTrainingEndpoint]", *a, flush=True)

    def _model_payload(self, fmt: bytes) -> bytes:
        blob = self.service.store.latest()
        if blob is None:
            return b"ERROR: no model"
        return blob.encode() if fmt == FMT_RRLM else blob.torchscript()

    def _listen_agents(self):
        while not self._stop.is_set():
            msg = self.router.recv(100)
            if msg is None:
                continue
            peer, frames = msg
            body = [f for f in frames if f != b""]
            if not body:
                continue
            cmd = body[0]
            try:
                if cmd == b"GET_MODEL":
                    fmt = body[1] if len(body) > 1 else FMT_TORCHSCRIPT
                    with self._lock:
                        if len(body) > 1:
                            self.agents[peer] = fmt
                        else:  # reference agent: updates go to its bound PULL, not the ROUTER
                            self.ref_agents.add(peer)
                            self._ref_push_dead = False
                            self._ref_push_failures = 0
                    self.service.register_agent(peer.decode(errors="replace"),
                                                None if len(body) > 1 else {"exempt": True, "reference": True})
                    self.router.send([peer, b"", self._model_payload(fmt)], 5000)
                elif cmd == b"MODEL_SET":
                    self.service.register_agent(peer.decode(errors="replace"))
                    self.router.send([peer, b"", b"ID_LOGGED"], 5000)
                    self._log("registered", peer)
                elif cmd == b"HEARTBEAT":
                    self.service.register_agent(peer.decode(errors="replace"))
                    with self._lock:  # an evicted agent that is alive again gets pushes again
                        if len(body) > 1 and peer not in self.agents:
                            self.agents[peer] = body[1]
                elif cmd == b"BYE":
                    with self._lock:
                        self.agents.pop(peer, None)
                else:
                    self.router.send([peer, b"", b"ERROR: unknown command"], 1000)
            except Exception as e:
                self._log("listener error", e)

    def _listen_traj(self):
        """Receive -> decode -> (in arrival order) dedupe + submit.  Reference frames are decoded
        to columns by C++ with the GIL released (ref_columns.h), on ``decode_threads`` workers
        at once; the ordered second stage keeps each agent's cumulative re-sends in sequence for
        the deduper."""
        from collections import deque

        pend = deque()  # (frame, future of its stage-1 decode or None)
        while not self._stop.is_set():
            msg = self.pull.recv(0 if pend else 100)
            if msg is not None:
                for f in msg[1]:
                    fut = self._decoders.submit(self._decode_stage1, f) if self._is_reference(f) else None
                    pend.append((f, fut))
            # finish in order: everything already decoded, or (no new input) wait for the head
            while pend and (pend[0][1] is None or pend[0][1].done() or msg is None):
                f, fut = pend.popleft()
                try:
                    traj = self._decode_traj(f, None if fut is None else fut.result())
                except Exception as e:
                    self.bad_frames += 1
                    self._log("bad trajectory frame", e)
                    continue
                if traj is not None:
                    self.service.submit(traj)

    @staticmethod
    def _is_reference(f: bytes) -> bool:
        from . import serde_pickle

        return not TrajectoryColumns.is_frame(f) and serde_pickle.is_pickle_frame(f)

    @staticmethod
    def _decode_stage1(f: bytes):
        """Worker thread: a reference frame to columns (GIL released inside), or the exception
        that sends it down the per-action path."""
        try:
            return ReferenceColumns.decode(f)
        except ValueError as e:
            return e

    def _decode_traj(self, f: bytes, cols=None):
        from . import serde_pickle

        if TrajectoryColumns.is_frame(f):
            return TrajectoryColumns.decode(f)
        if serde_pickle.is_pickle_frame(f):
            self.reference_frames += 1
            self._touch_reference_agents()
            if cols is None:
                cols = self._decode_stage1(f)
            if not isinstance(cols, Exception):  # natively, straight to columns
                rows = self.dedupe.new_rows(cols)
                return rows if len(rows) else None
            # ragged tensors / unusual encodings: the per-action path
            acts = self.dedupe.new_actions(serde_pickle.actions_from_reference(serde_pickle.loads_fast(f)))
            if not acts:
                return None
            t = RelayRLTrajectory(max(len(acts), 1), None, "reference-agent")
            t.actions = acts
            return t
        return RelayRLTrajectory.decode(f)

    def _on_model(self, blob: ModelBlob):
        """Publisher thread (LatestWorker): one blob, the newest, at a time."""
        with self._lock:
            agents = list(self.agents.items())
            push_ref = bool(self.ref_agents) and self.model_push_addr is not None and not self._ref_push_dead
        enc = {}
        for peer, fmt in agents:  # our agents first: an RRLM frame is a memcpy, no export
            if fmt not in enc:
                enc[fmt] = blob.encode() if fmt == FMT_RRLM else blob.torchscript()
            self.router.send([peer, b"", b"MODEL", str(blob.version).encode(), enc[fmt]], 1000)
        if push_ref:
            self._push_reference(blob)

    def _push_reference(self, blob: ModelBlob):
        """One TorchScript frame to the reference agents' bound PULL (agent_zmq.rs:625-698),
        built once per version.  A PUSH with no peer waits for one: after
        ``ref_push_max_failures`` consecutive timeouts the route is dropped -- the reference
        agents are unregistered from the learner -- until a GET_MODEL or a reference upload
        shows one is alive again."""
        if self._model_push is None:
            self._model_push = _native.ZmtpSocket(_native.SockType.PUSH)
            self._model_push.connect(self.model_push_addr)
        if self._model_push.send([blob.torchscript()], self.ref_push_timeout_ms):
            self.ref_pushes += 1
            with self._lock:
                self._ref_push_failures = 0
            return
        self.ref_push_timeouts += 1
        self._log("model push to", self.model_push_addr, "timed out")
        with self._lock:
            self._ref_push_failures += 1
            if self._ref_push_failures < self.ref_push_max_failures:
                return
            self._ref_push_dead = True
            gone = [p.decode(errors="replace") for p in self.ref_agents]
            self.ref_agents.clear()
        if hasattr(self.service, "forget_agents"):
            self.service.forget_agents(gone)
        self._log("reference push route dropped after", self.ref_push_max_failures, "failed sends:", gone)

    def flush(self, timeout_s: float = 10.0) -> bool:
        """Wait until the newest published model has been handed to every route."""
        return self._publisher.flush(timeout_s)

    def close(self):
        self._stop.set()
        self.service.store.unsubscribe(self._publisher)
        self._publisher.close()
        for t in self._threads:
            t.join(timeout=5)
        self._decoders.shutdown(wait=False)
        self.router.close()
        self.pull.close()
        if self._model_push is not None:
            self._model_push.close()


class ZmqAgentTransport:
    """DEALER handshake + model-update listener + PUSH trajectory sender."""

    def __init__(self, agent_id: str, agent_listener: str, trajectory_server: str,
                 on_model: Callable[[ModelBlob], None], handshake_timeout_s: float = 60.0,
                 heartbeat_s: float = 10.0):
        self.agent_id = agent_id
        self.on_model = on_model
        self.dealer = _native.ZmtpSocket(_native.SockType.DEALER, agent_id.encode())
        self.dealer.connect(agent_listener)
        self.push = _native.ZmtpSocket(_native.SockType.PUSH)
        self.push.connect(trajectory_server)
        self._replies = []
        self._cv = threading.Condition()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._recv_loop, daemon=True, name="rrl-agent-dealer")
        self._thread.start()
        self.model: Optional[ModelBlob] = None
        self._handshake(handshake_timeout_s)
        self._hb = None
        if heartbeat_s > 0:  # keeps an idle agent registered (LearnerService.start_sweeper)
            self._hb = threading.Thread(target=self._heartbeat_loop, args=(heartbeat_s,), daemon=True,
                                        name="rrl-agent-heartbeat")
            self._hb.start()

    def _heartbeat_loop(self, period_s: float):
        while not self._stop.wait(period_s):
            self.heartbeat()

    def _recv_loop(self):
        while not self._stop.is_set():
            msg = self.dealer.recv(100)
            if msg is None:
                continue
            _, frames = msg
            body = [f for f in frames if f != b""] if frames and frames[0] == b"" else frames
            if len(body) >= 3 and body[0] == b"MODEL":
                try:
                    blob = ModelBlob.decode(body[2])
                    self.model = blob
                    self.on_model(blob)
                except Exception as e:
                    print(f"[ZmqAgentTransport] bad model update: {e!r}", flush=True)
                continue
            with self._cv:
                self._replies.append(body)
                self._cv.notify_all()

    def _request(self, frames, timeout_s: float):
        with self._cv:
            self._replies.clear()
        if not self.dealer.send([b""] + frames, int(timeout_s * 1000)):
            return None
        with self._cv:
            self._cv.wait_for(lambda: bool(self._replies), timeout=timeout_s)
            return self._replies.pop(0) if self._replies else None

    def _handshake(self, timeout_s: float):
        """GET_MODEL -> MODEL_SET -> ID_LOGGED, retried every second (agent_zmq.rs:316-442)."""
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            rep = self._request([b"GET_MODEL", FMT_RRLM], 1.0)
            if rep and rep[0][:4] == b"RRLM":
                blob = ModelBlob.decode(rep[0])
                self.model = blob
                self.on_model(blob)
                ack = self._request([b"MODEL_SET"], 5.0)
                if ack and ack[0] == b"ID_LOGGED":
                    return
            time.sleep(0.05)
        raise TimeoutError("ZMQ handshake with the training server timed out")

    def send_trajectory(self, payload: bytes) -> bool:
        from ..utils.faults import injector

        payload = injector().filter_upload(payload)
        if payload is None:
            return True  # injected loss: the learner detects the sequence gap
        return self.push.send([payload], 10000)

    def heartbeat(self):
        self.dealer.send([b"", b"HEARTBEAT", FMT_RRLM], 1000)

    def close(self):
        try:
            self.dealer.send([b"", b"BYE"], 200)
        except Exception:
            pass
        self._stop.set()
        self._thread.join(timeout=5)
        if self._hb is not None:
            self._hb.join(timeout=5)
        self.dealer.close()
        self.push.close()


class ReferenceZmqAgentTransport:
    """The reference agent's own wire, for talking to a reference (Rust) training server
    (or to ZmqTrainingEndpoint, which accepts both dialects):

      * handshake (agent_zmq.rs:316-442): DEALER (identity = agent id) -> ``["", "GET_MODEL"]``
        with NO format frame; the server answers ``["", <TorchScript archive>]`` (or
        ``"ERROR: ..."``); the agent loads it, then ``["", "MODEL_SET"]`` -> ``["", "ID_LOGGED"]``;
        retried every second until the timeout;
      * uploads (trajectory.rs:50-90): ``serde_pickle(Vec<RelayRLAction>)`` frames on a PUSH to
        ``trajectory_server`` -- one connection for all uploads, or, with
        ``connection_per_upload``, a new connection + handshake per upload exactly like the
        reference agent (its new zmq context + PUSH per send; the server's fan-in test case);
      * model updates (agent_zmq.rs:625-698): the agent BINDS a PULL on its ``training_server``
        address and the server PUSH-connects to it, one TorchScript archive per update.  A
        receive thread blocks with a timeout (no busy poll) and swaps the policy.
    Archives are read by ``utils.checkpoint.reference_weights_from_bytes`` (raw zip storages;
    nothing in them is unpickled or executed)."""

    def __init__(self, agent_id: str, agent_listener: str, trajectory_server: str, training_server: str,
                 on_model: Callable[[ModelBlob], None], handshake_timeout_s: float = 60.0,
                 connection_per_upload: bool = False):
        self.agent_id = agent_id
        self.on_model = on_model
        self.version = 0
        self.bad_models = 0
        self.trajectory_server = trajectory_server
        self.connection_per_upload = bool(connection_per_upload)
        self.pull = _native.ZmtpSocket(_native.SockType.PULL)
        self.pull.bind(training_server)  # before the handshake: the server may push at once
        self.dealer = _native.ZmtpSocket(_native.SockType.DEALER, agent_id.encode())
        self.dealer.connect(agent_listener)
        self.push = _native.ZmtpSocket(_native.SockType.PUSH)
        self.push.connect(trajectory_server)
        self._stop = threading.Event()
        self._handshake(handshake_timeout_s)
        self._thread = threading.Thread(target=self._model_loop, daemon=True, name="rrl-ref-agent-models")
        self._thread.start()

    def _load(self, blob: bytes) -> ModelBlob:
        from ..runtime.model_store import blob_from_archive

        mb = blob_from_archive(self.version + 1, blob)
        self.on_model(mb)  # raises if the agent cannot validate it (the version is not taken)
        self.version += 1
        return mb

    def _recv_reply(self, timeout_s: float):
        msg = self.dealer.recv(int(timeout_s * 1000))
        if msg is None:
            return None
        _, frames = msg
        body = [f for f in frames if f != b""]
        return body[0] if body else None

    def _handshake(self, timeout_s: float):
        t0 = time.time()
        while time.time() - t0 < timeout_s:
            if not self.dealer.send([b"", b"GET_MODEL"], 1000):
                time.sleep(1.0)
                continue
            rep = self._recv_reply(2.0)
            if rep is None or rep.startswith(b"ERROR"):
                time.sleep(1.0)  # agent_zmq.rs retries every second
                continue
            try:
                self._load(rep)
            except Exception as e:  # a model the agent cannot validate: ask again
                self.bad_models += 1
                print(f"[ReferenceZmqAgentTransport] bad model in the handshake: {e!r}", flush=True)
                time.sleep(1.0)
                continue
            if self.dealer.send([b"", b"MODEL_SET"], 1000) and self._recv_reply(5.0) == b"ID_LOGGED":
                return
        raise TimeoutError("reference ZMQ handshake with the training server timed out")

    def _model_loop(self):
        while not self._stop.is_set():
            msg = self.pull.recv(100)
            if msg is None:
                continue
            _, frames = msg
            for f in frames:
                if not f:
                    continue
                try:
                    self._load(f)
                except Exception as e:
                    self.bad_models += 1
                    print(f"[ReferenceZmqAgentTransport] bad model update: {e!r}", flush=True)

    def send_trajectory(self, payload: bytes) -> bool:
        from ..utils.faults import injector

        payload = injector().filter_upload(payload)
        if payload is None:
            return True
        if self.connection_per_upload:
            s = _native.ZmtpSocket(_native.SockType.PUSH)
            try:
                s.connect(self.trajectory_server)
                return s.send([payload], 10000)
            finally:
                s.close()
        return self.push.send([payload], 10000)

    def heartbeat(self):
        pass  # the reference protocol has none (the server exempts reference agents from eviction)

    def close(self):
        self._stop.set()
        self._thread.join(timeout=5)
        self.dealer.close()
        self.push.close()
        self.pull.close()
